# round 5: the share lanes-per-pixel sweep (gpu_r05k.sh), then the steady-state PMC records and same-box forecast
bash scripts/gpu_r05k.sh && bash scripts/gpu_r05_pmc.sh r05p
