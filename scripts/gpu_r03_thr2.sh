# Secondary-round threshold on RTWeekend after the REL member rule (RT_SEC_THRESHOLD; default 40 there).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  bash scripts/gpu_ab_cfg.sh rtw 3 "RT_X=0" "RT_SEC_THRESHOLD=32" "RT_SEC_THRESHOLD=48" "RT_SEC_THRESHOLD=56" || exit 1
done
