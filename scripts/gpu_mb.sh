set -o pipefail
mkdir -p gpurun_out
for args in "4 8192 20000" "2 8192 20000"; do
  timeout -k 10 120 ./scripts/mb_valu $args || exit $?
done
