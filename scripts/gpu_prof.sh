# needs scripts/mb_valu: hipcc --offload-arch=gfx950 -O3 scripts/mb_valu.hip -o scripts/mb_valu (built here, travels to the box)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 120 ./scripts/mb_valu > gpurun_out/mb_valu.log 2>&1 || exit $?
cat gpurun_out/mb_valu.log
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc1 -o p1 --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VALU -d gpurun_out/pmc2 -o p2 --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3 -o p3 --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc4 -o p4 --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc4.log 2>&1 || exit $?
ls gpurun_out/pmc*
