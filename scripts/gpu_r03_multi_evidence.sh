# Round-3 multi-device evidence on one GPU: OnRender over two device slots, the
# single-process rt_multi bench at 3 shares, a kernel + copy trace of rt_multi over
# eight shares (gather and assembly cost, cold-call overlap across devices), and the
# refreshed 2- and 4-rank forecast rows.
set -o pipefail
mkdir -p gpurun_out
BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --config onrender --gpus 2 --frames 128 > gpurun_out/me_onrender.json 2> gpurun_out/me.err || { tail -5 gpurun_out/me.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/me_onrender.json'))
for r in d['runs']: print(json.dumps(r))"
BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 3 --steps 5 --warmup 3 > gpurun_out/me_g3.json 2> gpurun_out/me.err || { tail -5 gpurun_out/me.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/me_g3.json')); print({k: d[k] for k in ('value','ms_per_step','per_device_trace_ms','call_ms_events','one_gpu','verified','cold_ms')})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BENCH_SHARE_GPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/me_kt -o run --output-format csv -- python3 bench.py --gpus 8 --steps 3 --warmup 2 --no-verify > gpurun_out/me_kt.log 2>&1 || { tail -5 gpurun_out/me_kt.log; exit 1; }
tail -c 300 gpurun_out/me_kt.log; echo
for g in 2 4; do echo "== $g ranks"; bash scripts/gpu_simranks_all.sh $g || exit 1; done
for spec in "2 16" "4 16"; do
  set -- $spec
  RT_LANES_PER_PIXEL=$2 timeout -k 10 120 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --sim-ranks $1 --sim-index 0 2> gpurun_out/fc.err | tail -1 | sed "s/^/P=$2 /" || { tail -5 gpurun_out/fc.err; exit 1; }
done
