# instrumented library for tools/diag/qt_prof.py: orb-slam-_amd/build_prof/liborbx.so built with -DORBX_QT_PROF
#   bash tools/diag/build_prof.sh   (on the CPU, before the GPU call)
set -e
cd "$(dirname "$0")/../../orb-slam-_amd"
mkdir -p build_prof
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -DORBX_QT_PROF"
for s in csrc/*.hip; do /opt/rocm/bin/hipcc $F -c $s -o build_prof/$(basename $s .hip).o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_prof/liborbx.so build_prof/*.o
