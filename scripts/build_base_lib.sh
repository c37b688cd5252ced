# Builds librt_trace_<name>.so from the kernel source at a git revision (default HEAD),
# with the working tree's host objects, for same-box A/B runs (RT_TRACE_LIB=...).
# usage: bash scripts/build_base_lib.sh [rev] [name]
set -e
rev=${1:-HEAD}; name=${2:-base}
cd "$(dirname "$0")/../simd-ray-tracer_amd"
make -s build/rt_host.o build/rt_scene.o build/rt_app.o build/rt_image.o build/rt_multi.o
git show "$rev:simd-ray-tracer_amd/csrc/rt_kernel.hip" > build/rt_kernel_$name.hip
git show "$rev:simd-ray-tracer_amd/csrc/rt_kernel.h" > build/rt_kernel_$name.h
sed -i "s/#include \"rt_kernel.h\"/#include \"rt_kernel_$name.h\"/" build/rt_kernel_$name.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Icsrc -Ibuild \
  -fno-slp-vectorize $KFLAGS -c build/rt_kernel_$name.hip -o build/rt_kernel_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o librt_trace_$name.so build/rt_kernel_$name.o build/rt_host.o \
  build/rt_scene.o build/rt_app.o build/rt_image.o build/rt_multi.o -ldl
echo "built librt_trace_$name.so from $rev"
