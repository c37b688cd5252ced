# round 5: heavy-wave spreading with priority (RT_HEAVY_SPREAD / RT_HEAVY_COUNT) on C2 and the 8-rank share,
# then the share lanes-per-pixel sweep (gpu_r05k.sh)
VARIANTS="RT_X=0;RT_HEAVY_SPREAD=7 RT_HEAVY_COUNT=128;RT_HEAVY_SPREAD=4 RT_HEAVY_COUNT=128;RT_HEAVY_SPREAD=7 RT_HEAVY_COUNT=48" \
CONFIGS="c2;--sim-ranks 8 --sim-index 0;--config rtw" ROUNDS=2 bash scripts/gpu_ab.sh && bash scripts/gpu_r05k.sh
