# PMC passes over one bench launch (kernel-trace counters only, no sys-trace).
# usage: bash scripts/gpu_pmc.sh <tag> [extra bench args]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE" "SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_IFETCH SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/pmc_${tag}_$i -o p --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pmc_${tag}_$i.log 2>&1 || exit $?
done
python scripts/pmc_summary.py gpurun_out pmc_${tag}_ > gpurun_out/pmc_${tag}_summary.txt
cat gpurun_out/pmc_${tag}_summary.txt
