# Builds librt_trace_<name>.so from the whole library source at a git revision
# (default HEAD) -- its own kernel translation units, host objects, header and
# Makefile, exported into a scratch directory -- for same-box A/B runs
# (RT_TRACE_LIB=librt_trace_<name>.so).  KFLAGS (optional) are passed to the
# revision's kernel build when its Makefile has the `variant` target.
# usage: bash scripts/build_base_lib.sh [rev] [name]
set -e
rev=${1:-HEAD}; name=${2:-base}
repo="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d /tmp/rt_base_XXXXXX)
git -C "$repo" archive "$rev" simd-ray-tracer_amd include | tar -x -C "$tmp"
if [ -n "$KFLAGS" ]; then
  make -s -j8 -C "$tmp/simd-ray-tracer_amd" variant NAME="$name" KFLAGS="$KFLAGS"
  cp "$tmp/simd-ray-tracer_amd/librt_trace_$name.so" "$repo/simd-ray-tracer_amd/librt_trace_$name.so"
else
  make -s -j8 -C "$tmp/simd-ray-tracer_amd" librt_trace.so
  cp "$tmp/simd-ray-tracer_amd/librt_trace.so" "$repo/simd-ray-tracer_amd/librt_trace_$name.so"
fi
# every symbol must resolve (a revision whose Makefile links no P = 16 object would leave rtk_launch_p16 undefined)
if nm -D --undefined-only "$repo/simd-ray-tracer_amd/librt_trace_$name.so" | grep -q " rtk_"; then
  echo "librt_trace_$name.so has undefined rtk_ symbols" >&2; exit 1
fi
rm -rf "$tmp"
echo "built librt_trace_$name.so from $rev"
