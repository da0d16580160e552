# As build_variant.sh, without refreshing the regular build first: attn_bf16.hip and capi.hip
# compiled with the extra flags, linked with the build/*.o already there (A/B variants whose
# other units do not matter, e.g. bf16 kernels limited to a few configs by DTA_FOR_CONFIGS).
#   bash tools/build_variant_fast.sh <name> "<flags>"
set -e
NAME=$1; EXTRA=$2
C=$(dirname $0)/../differential_transformer_replication_amd/csrc
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -fno-honor-nans -fno-slp-vectorize -w"
mkdir -p $C/build_v
/opt/rocm/bin/hipcc $FLAGS $EXTRA -c ${SRC:-$C/attn_bf16.hip} -o $C/build_v/attn_bf16_$NAME.o
/opt/rocm/bin/hipcc $FLAGS $EXTRA -c $C/capi.hip -o $C/build_v/capi_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $C/build_v/capi_$NAME.o $C/build/elementwise.o $C/build/decode.o \
  $C/build/attn_f16.o $C/build/attn_f32.o $C/build/attn_bf16_drop.o $C/build/attn_f16_drop.o $C/build/attn_f32_drop.o $C/build_v/attn_bf16_$NAME.o -o $C/../lib/libdiffattn_$NAME.so
echo built lib/libdiffattn_$NAME.so
