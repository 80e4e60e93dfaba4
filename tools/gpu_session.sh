# same-box A/B: working tree vs HEAD (pre) vs round-5 end (r05): per-layer C5 AE times + step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
sed -i 's/timeout -k 10 120 python/timeout -k 10 200 python/' tools/lib_ab.sh
timeout -k 10 600 bash tools/lib_ab.sh tools/layer_ab.py --reps 20 -- main pre r05 > gpurun_out/s11_layer_ab.txt 2>&1 || { tail -20 gpurun_out/s11_layer_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s11_layer_ab.txt | tail -40
timeout -k 10 600 bash tools/lib_ab.sh bench.py --steps 30 --warmup 5 --no-stages --no-cpu-baseline -- main pre r05 > gpurun_out/s11_bench_ab.txt 2>&1 || { tail -20 gpurun_out/s11_bench_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s11_bench_ab.txt | python -c "
import sys, json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('=='): print(l, end=' ')
    elif l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'])
"
