# an alternative build of liborbx.so for A/B runs (loaded with ORBX_LIB=orb-slam-_amd/DIR/liborbx.so)
#   bash tools/diag/build_alt.sh DIR -DFLAG=...   (on the CPU, before the GPU call)
set -e
D=$1; shift
cd "$(dirname "$0")/../../orb-slam-_amd"
mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w $*"
for s in csrc/*.hip; do /opt/rocm/bin/hipcc $F -c $s -o $D/$(basename $s .hip).o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/liborbx.so $D/*.o
