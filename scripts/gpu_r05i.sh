# round 5: XCD-grouping check and A/B (gpu_r05h.sh), then part 1 of the round evidence
bash scripts/gpu_r05h.sh && bash scripts/gpu_r05_evidence.sh r05 1
