set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for b in 1 2 8; do
  RT_SEC_THRESHOLD=16 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/pmcb$b -o p --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --bounces $b > gpurun_out/pmcb$b.log 2>&1 || exit $?
  echo "bounces $b"; python scripts/pmc_summary.py gpurun_out pmcb$b
done
