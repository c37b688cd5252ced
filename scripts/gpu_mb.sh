set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for args in "4 8192 100000 0" "4 2048 100000 0" "4 2048 20000 0" "4 8192 20000 0" "4 4096 20000 0" "4 16384 20000 0" "4 2048 20000 3" "4 8192 20000 3" "4 8192 20000 5"; do
  timeout -k 10 120 ./scripts/mb_valu $args || exit $?
done
