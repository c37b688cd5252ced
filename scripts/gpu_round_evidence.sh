# Round evidence, in two GPU calls (each step under its own timeout, chained so a failure stops the call):
#   bash scripts/gpu_round_evidence.sh <tag> suite   GPU suite, smoke(), the driver's default bench line, the
#                                                    rocprofv3 kernel trace + --stats of that same command, the
#                                                    other configurations' lines (C3, RTWeekend, C2-inside, C5,
#                                                    C5's one-box 8-way split, the brute-force kernel)
#   bash scripts/gpu_round_evidence.sh <tag> pmc     the PMC records (scripts/gpu_pmc.sh -> pmc_to_json.py, each
#                                                    stamped with the library's code-object hash): C2, C2
#                                                    brute force, RTWeekend, C3, C5, the 2/4/8-rank shares of C2
#                                                    (residue 0) and the OnRender 1-spp frame
# Writes gpurun_out/ev_<tag>_*; copy what is judged into profiles/.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-ev}
part=${2:-suite}
W=gpurun_out/ev_${tag}
if [ "$part" = suite ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    > ${W}_pytest.log 2>&1 || { tail -20 ${W}_pytest.log; exit 1; }
  tail -1 ${W}_pytest.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > ${W}_smoke.log 2>&1 || { tail -5 ${W}_smoke.log; exit 1; }
  tail -1 ${W}_smoke.log
  timeout -k 10 300 python bench.py > ${W}_bench.json 2> ${W}_bench.err || { tail -5 ${W}_bench.err; exit 1; }
  tail -c 300 ${W}_bench.json; echo
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${W}_trace -o run --output-format csv -- python bench.py \
    > ${W}_trace.log 2>&1 || { tail -5 ${W}_trace.log; exit 1; }
  # the headline's timed launches alone (--legs none): the last 5 dispatches of its kernel are the 5 timed steps
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${W}_trace_headline -o run --output-format csv -- python bench.py \
    --legs none --no-cpu-baseline > ${W}_trace_headline.log 2>&1 || { tail -5 ${W}_trace_headline.log; exit 1; }
  f=$(find ${W}_trace_headline -name "*kernel_trace.csv" | head -1)
  python scripts/kernel_timeline.py "$f" --tail 5 --kernel "trace_kernel<true, 0, true" > ${W}_timeline.txt || exit 1
  for cfg in c3 rtw c2in; do
    timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 3 --no-cpu-baseline --legs distinct \
      >> ${W}_configs.jsonl 2>> ${W}_configs.err || exit 1
  done
  timeout -k 10 300 python bench.py --brute --steps 5 --warmup 3 --no-cpu-baseline --legs none >> ${W}_configs.jsonl \
    2>> ${W}_configs.err || exit 1
  timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 2 --no-cpu-baseline --legs none >> ${W}_configs.jsonl \
    2>> ${W}_configs.err || exit 1
  BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --config c5 --gpus 8 --steps 1 --warmup 2 >> ${W}_configs.jsonl \
    2>> ${W}_configs.err || exit 1
  echo suite done
elif [ "$part" = pmc ]; then
  C2="C2: 1920x1080, 256 spp, 64 spheres, 8 bounces, SIMD rules"
  run() {  # run <name> <workload> <bands> [bench args]
    local name=$1 wl=$2 bands=$3; shift 3
    bash scripts/gpu_pmc.sh ${tag}${name} "$@" > ${W}_${name}_pmc_stdout.txt 2>&1 || { tail -5 ${W}_${name}_pmc_stdout.txt; return 1; }
    python scripts/pmc_to_json.py gpurun_out pmc_${tag}${name}_ ${W}_${name}_pmc.json "$wl" $bands > /dev/null || return 1
    python scripts/pmc_brief.py ${W}_${name}_pmc.json
  }
  run c2 "$C2" 1 || exit 1
  run c2brute "$C2 [Cull=-1, Prefilter=-1]" 1 --brute || exit 1
  run rtw "RTW: 1920x1080, 64 spp, 482 spheres, 8 bounces, SIMD rules, RTWeekend" 1 --config rtw || exit 1
  run c3 "C3: 3840x2160, 1024 spp, 64 spheres, 8 bounces, SIMD rules" 1 --config c3 || exit 1
  PMC_WARMUP=4 run c5 "C5: 7680x4320, 4096 spp, 256 spheres, 16 bounces, SIMD rules" 1 --config c5 || exit 1
  for g in 2 4 8; do
    run c2rank$g "$C2" $g --sim-ranks $g --sim-index 0 || exit 1
  done
  run onrender "onrender_static_1080p" 1 --config onrender --width 1920 --height 1080 --modes static --frames 128 || exit 1
  echo pmc done
fi
