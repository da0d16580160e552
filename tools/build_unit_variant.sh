# Build lib/libdiffattn_<name>.so with ONE translation unit recompiled with extra flags
# (everything else from the regular build):
#   bash tools/build_unit_variant.sh <name> <unit> "<flags>"     e.g. v3 attn_bf16_dq2 "-DDTA_DQ2_R=3"
set -e
NAME=$1; UNIT=$2; EXTRA=$3
C=$(dirname $0)/../differential_transformer_replication_amd/csrc
make -C $C -j8 >/dev/null
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -fno-honor-nans -fno-slp-vectorize -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-but-set-variable"
[ "$UNIT" = attn_bf16_dq2 ] && FLAGS="$FLAGS -mllvm -amdgpu-mfma-vgpr-form=1"
mkdir -p $C/build_v
/opt/rocm/bin/hipcc $FLAGS $EXTRA -c $C/$UNIT.hip -o $C/build_v/${UNIT}_$NAME.o
OBJS=$(ls $C/build/*.o | grep -v "/$UNIT.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $C/build_v/${UNIT}_$NAME.o -o $C/../lib/libdiffattn_$NAME.so
echo built lib/libdiffattn_$NAME.so
