# needs scripts/mb_valu: hipcc --offload-arch=gfx950 -O3 scripts/mb_valu.hip -o scripts/mb_valu (built here, travels to the box)
set -o pipefail
mkdir -p gpurun_out
for args in "4 8192 20000" "2 8192 20000"; do
  timeout -k 10 120 ./scripts/mb_valu $args || exit $?
done
