# Instruction counts and VALU occupancy of C2 with and without deferred shading (same box).
set -o pipefail
RT_TRACE_LIB=librt_trace.so bash scripts/gpu_pmc_quick.sh nodefer "" || exit $?
RT_TRACE_LIB=librt_trace_defer.so bash scripts/gpu_pmc_quick.sh defer "" || exit $?
