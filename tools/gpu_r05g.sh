R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/lib_ab.sh tools/stft_c2_bench.py -- main nt2 sc1 sc01 > gpurun_out/stft_ab_r05g.txt 2>&1 || { tail -20 gpurun_out/stft_ab_r05g.txt; exit 1; }
grep -v amdgpu gpurun_out/stft_ab_r05g.txt
