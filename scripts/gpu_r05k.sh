# round 5: lanes per pixel of the 2/4/8-rank shares re-swept at the final kernel, with the whole frame on the same box
VARIANTS="RT_X=0;RT_LANES_PER_PIXEL=4;RT_LANES_PER_PIXEL=8;RT_LANES_PER_PIXEL=16" \
CONFIGS="c2;--sim-ranks 8 --sim-index 0;--sim-ranks 4 --sim-index 0;--sim-ranks 2 --sim-index 0" ROUNDS=2 bash scripts/gpu_ab.sh
