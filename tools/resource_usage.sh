# Per-kernel VGPR / scratch / occupancy of the attention kernels (cross-compiled, no GPU).
cd $(dirname $0)/../differential_transformer_replication_amd/csrc
for f in ${@:-attn_bf16 attn_f16 attn_f32}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -fno-honor-nans -fno-slp-vectorize \
    -Rpass-analysis=kernel-resource-usage -c $f.hip -o /dev/null 2>&1 | python3 -c "
import sys, re
name = None; row = {}
for l in sys.stdin:
    m = re.search(r'Function Name: (\S+)', l)
    if m: name = m.group(1); row = {}
    for key in ('VGPRs', 'AGPRs', 'ScratchSize \[bytes/lane\]', 'Occupancy \[waves/SIMD\]', 'LDS Size \[bytes/block\]'):
        m = re.search(key + r': (\d+)', l)
        if m: row[key.split()[0]] = int(m.group(1))
    if name and 'LDS' in row:
        n = re.sub(r'_ZN3dta\d+', '', name).replace('EEEvNS_9', ' ').replace('Params', '')
        print(f'{n[:64]:64s} v{row.get(\"VGPRs\")} a{row.get(\"AGPRs\")} scr{row.get(\"ScratchSize\")} occ{row.get(\"Occupancy\")}')
        name = None
"
done
