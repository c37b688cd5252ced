# round 5: exact-sequence check, GPU suite + C2/RTW lines, pixel-segment A/B, writes
timeout -k 10 120 ./scripts/mathcheck > gpurun_out/r05b_mathcheck.txt 2>&1; cat gpurun_out/r05b_mathcheck.txt
bash scripts/gpu_check.sh r05b --configs "rtw" && \
VARIANTS="RT_PIXEL_SEG=1;RT_PIXEL_SEG=4" CONFIGS="c2;--config rtw" ROUNDS=2 bash scripts/gpu_ab.sh && \
VARIANTS="RT_PIXEL_SEG=1;RT_PIXEL_SEG=4" CONFIGS="c2;--config rtw" bash scripts/gpu_writes.sh
