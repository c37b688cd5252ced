# round 5: pixel-segment size with the RGBA8 encode pass on (default): A/B and trace-kernel HBM bytes
VARIANTS="RT_PIXEL_SEG=1;RT_PIXEL_SEG=2;RT_PIXEL_SEG=4" CONFIGS="c2;--config rtw" ROUNDS=2 bash scripts/gpu_ab.sh && \
VARIANTS="RT_PIXEL_SEG=1;RT_PIXEL_SEG=2;RT_PIXEL_SEG=4" CONFIGS="c2;--config rtw" bash scripts/gpu_writes.sh
