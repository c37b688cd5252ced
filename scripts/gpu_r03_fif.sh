# Frames in flight: two rt_device contexts on one GPU tracing alternate frames (C2, the 8-rank share).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/frames_in_flight.py 16 2 || exit 1
timeout -k 10 200 python scripts/frames_in_flight.py 16 3 || exit 1
timeout -k 10 200 python scripts/frames_in_flight.py 40 2 --sim-ranks 8 --sim-index 3 || exit 1
timeout -k 10 200 python scripts/frames_in_flight.py 40 2 --sim-ranks 4 --sim-index 0 || exit 1
