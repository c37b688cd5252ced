# round 5: issue-priority A/B (RT_PRIO_PERMILLE, RT_PRIO_DRAIN) on C2, RTWeekend and the 8-rank share
VARIANTS="RT_X=0;RT_PRIO_PERMILLE=125;RT_PRIO_PERMILLE=300;RT_PRIO_DRAIN=1" CONFIGS="c2;--config rtw;--sim-ranks 8 --sim-index 3" ROUNDS=2 bash scripts/gpu_ab.sh
