# One-wave kernels at 8 waves/SIMD now that their cull mask is dynamic LDS (4352 B per
# workgroup instead of 4864): same-box A/B of HEAD (base), the default build and the w8 variant.
set -o pipefail
mkdir -p gpurun_out
LIBS="librt_trace_base.so librt_trace.so librt_trace_w8.so" ROUNDS=2 timeout -k 10 600 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="librt_trace_base.so librt_trace.so librt_trace_w8.so" ROUNDS=1 CONFIGS="--config rtw;--config c5 --spp 256" timeout -k 10 600 bash scripts/gpu_lib_ab.sh
