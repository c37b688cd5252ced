# Rehearsal of bench.py's multi-rank path on a 1-GPU box: N ranks (gloo, all on
# cuda:0) render their bands, gather to rank 0, assemble, and rank 0 verifies
# the assembled frame bit-for-bit against a one-rank render.
set -o pipefail
mkdir -p gpurun_out
for n in 2 3 8; do
  BENCH_BACKEND=gloo BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 3 --warmup 1 --verify \
    --width 640 --height 360 --spp 32 > gpurun_out/mr$n.json 2> gpurun_out/mr$n.err || { tail -20 gpurun_out/mr$n.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/mr$n.json') if l.startswith('{')][-1]); print('ranks $n', d['value'], d['ms_per_step'], 'verified', d.get('verified'))"
done
timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify --width 640 --height 360 --spp 32 > gpurun_out/mr1.json
python -c "import json; d=json.load(open('gpurun_out/mr1.json')); print('ranks 1', d['value'], d['ms_per_step'], 'verified', d.get('verified'))"
