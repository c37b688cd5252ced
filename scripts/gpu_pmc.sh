# PMC passes over the trace kernel (kernel-trace counters only, no sys-trace):
# bench.py --steps 1 --warmup 7 under each counter set (the timed launch is then past
# the order-learning launches: no wave/pixel cost stores, no sorts); scripts/pmc_to_json.py
# keeps the LAST trace_kernel dispatch of every pass (the warm launch the
# bench times, learned tile order in place).
# usage: bash scripts/gpu_pmc.sh <tag> [extra bench args]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_IFETCH GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc_${tag}_$i -o p --output-format csv -- python bench.py --steps 1 --warmup ${PMC_WARMUP:-7} --no-cpu-baseline --headline-only "$@" > gpurun_out/pmc_${tag}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${tag}_$i.log; exit 1; }
done
echo "pmc passes done: $i"
