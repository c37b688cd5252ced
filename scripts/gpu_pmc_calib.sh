# Which SQ counters count which gfx950 VALU instructions, and at what weight:
# scripts/mb_ops (hipcc --offload-arch=gfx950 -O3 scripts/mb_ops.hip -o scripts/mb_ops, built in
# the container) under rocprofv3 --pmc, one pass per counter set.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/cal_$i -o p --output-format csv -- ./scripts/mb_ops > gpurun_out/cal_$i.log 2>&1 || { tail -5 gpurun_out/cal_$i.log; exit 1; }
done
python scripts/pmc_calib.py gpurun_out cal_ | tee gpurun_out/pmc_calib.txt
