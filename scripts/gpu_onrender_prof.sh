# The reference's per-frame unit (OnRender, 1 spp per call) under rocprofv3:
# a kernel trace of the static 1080p loop (what each frame's GPU time goes
# to) and the PMC passes of scripts/gpu_pmc.sh over its trace kernel.
# usage: bash scripts/gpu_onrender_prof.sh <tag> [extra bench args]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
ARGS="--config onrender --width 1920 --height 1080 --modes static --frames 128 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_kt -o run --output-format csv -- python bench.py $ARGS > gpurun_out/${tag}_kt.log 2>&1 || { tail -5 gpurun_out/${tag}_kt.log; exit 1; }
f=$(find gpurun_out/${tag}_kt -name "*kernel_trace.csv" | head -1)
python scripts/kernel_timeline.py "$f" --tail 64 > gpurun_out/${tag}_timeline.txt || exit 1
cat gpurun_out/${tag}_timeline.txt
timeout -k 10 120 python bench.py $ARGS > gpurun_out/${tag}_bench.log 2>&1 || exit 1
tail -2 gpurun_out/${tag}_bench.log
bash scripts/gpu_pmc.sh ${tag} $ARGS || exit 1
python scripts/pmc_to_json.py gpurun_out pmc_${tag}_ gpurun_out/${tag}_pmc.json onrender_static_1080p && python scripts/pmc_brief.py gpurun_out/${tag}_pmc.json
