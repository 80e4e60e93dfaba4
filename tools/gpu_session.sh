set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 bash tools/lib_ab.sh tools/svd_c5.py -- main noswz > gpurun_out/s3_top1_ab.txt 2>&1 || { tail -5 gpurun_out/s3_top1_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s3_top1_ab.txt
timeout -k 10 300 bash tools/lib_ab.sh tools/stft_c5.py 4096 -- main nopad > gpurun_out/s3_stft_ab.txt 2>&1 || { tail -5 gpurun_out/s3_stft_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s3_stft_ab.txt
bash tools/gpu.sh s3 bench
