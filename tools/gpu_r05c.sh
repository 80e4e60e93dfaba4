cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/lib_ab.sh tools/stft_c2_bench.py -- main w8pf0 w8pf1 w4pf0 > gpurun_out/stft_ab_r05c.txt 2>&1 || { tail gpurun_out/stft_ab_r05c.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stft_ab_r05c.txt
for M in 3layer manual_scan hyper_k3 hyper_k5 hyper_k7; do
  timeout -k 10 120 python tools/ae_bench.py --model $M --dtype bf16 >> gpurun_out/ae_bench_r05c.txt 2>&1 || exit 1
done
for M in 3layer hyper_k3; do
  timeout -k 10 120 python tools/ae_bench.py --model $M --dtype float16 >> gpurun_out/ae_bench_r05c.txt 2>&1 || exit 1
done
R=$GRAFT_REPO_ROOT; TAG=r05c
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stages --streams 1 > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err || exit 1
mkdir -p $R/gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name '*stats.csv' -exec cp {} $R/gpurun_out/prof_$TAG/ \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profc4_$TAG -o prof -- python3 $R/tools/c4_prof.py --steps 30 > $R/gpurun_out/c4prof_$TAG.log 2>&1 || exit 1
mkdir -p $R/gpurun_out/profc4_$TAG && find /tmp/profc4_$TAG -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/profc4_$TAG/ \;
cd $R && bash tools/pmc_refresh.sh c5 c2 || exit 1
echo done
