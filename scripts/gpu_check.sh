# The GPU suite, then (only when it passes) the default C2 line and optional extra steps.
# usage: bash scripts/gpu_check.sh <tag> [--onrender] [--configs "rtw c5 ..."]
set -o pipefail
mkdir -p gpurun_out
tag=${1:-chk}; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/${tag}_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_c2.json 2> gpurun_out/${tag}_c2.err || { tail -5 gpurun_out/${tag}_c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${tag}_c2.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
while [ $# -gt 0 ]; do
  case $1 in
    --onrender)
      timeout -k 10 300 python bench.py --config onrender > gpurun_out/${tag}_onr.json 2> gpurun_out/${tag}_onr.err || { tail -5 gpurun_out/${tag}_onr.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/${tag}_onr.json')); [print('onrender', r['width'], r['mode'], r['mrays_per_s'], r['ms_per_frame'], r.get('gpu_ms_per_frame')) for r in d['runs']]"
      shift ;;
    --configs)
      for c in $2; do
        timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 3 --no-cpu-baseline >> gpurun_out/${tag}_configs.jsonl 2>> gpurun_out/${tag}_configs.err || { tail -5 gpurun_out/${tag}_configs.err; exit 1; }
        tail -1 gpurun_out/${tag}_configs.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
      done
      shift 2 ;;
    *) shift ;;
  esac
done
