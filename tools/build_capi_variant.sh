# Build lib/libdiffattn_<name>.so with capi.hip compiled with extra flags (e.g.
# -DDTA_BWD_GROUP_MAX=2), every kernel object from the regular build.
#   bash tools/build_capi_variant.sh <name> "<flags>"
set -e
NAME=$1; EXTRA=$2
C=$(dirname $0)/../differential_transformer_replication_amd/csrc
make -C $C -j8 >/dev/null
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -fno-honor-nans -fno-slp-vectorize -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-but-set-variable"
mkdir -p $C/build_v
/opt/rocm/bin/hipcc $FLAGS $EXTRA -c $C/capi.hip -o $C/build_v/capi_$NAME.o
OBJS=$(ls $C/build/*.o | grep -v '/capi.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $C/build_v/capi_$NAME.o $OBJS -o $C/../lib/libdiffattn_$NAME.so
echo built lib/libdiffattn_$NAME.so
