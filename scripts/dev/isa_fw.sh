#!/bin/bash
# gfx950 ISA of the fused sweep + the resource usage of one instance (default: the
# C3 bench instance rq_sweep_fw<1, uint16, 16, 8, BITS, !PW>).
# usage: scripts/dev/isa_fw.sh [OUT.s] [extra hipcc flags]
OUT=${1:-/tmp/isa/fw_all.s}; shift
INST=${INST:-_Z11rq_sweep_fwILi1EtLi16ELi8ELb1ELb0EEv9SweepArgs}
mkdir -p "$(dirname "$OUT")"
cd "$(dirname "$0")/../../redqueen_amd/csrc"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -std=c++17 "$@" \
  --cuda-device-only -S -o "$OUT" rq_sweep_fw.hip -Rpass-analysis=kernel-resource-usage 2> "$OUT.remarks"
awk -v n="$INST" '/Function Name:/{p=index($0,n)>0} p' "$OUT.remarks" | grep -E "VGPRs|SGPRs|Spill|Occupancy|ScratchSize" | sed 's/.*remark: *//'
python3 - "$OUT" "$INST" <<'PY'
import re, sys
L = open(sys.argv[1]).read().split('\n')
name = sys.argv[2] + ':'
s = [i for i, l in enumerate(L) if l.startswith(name)][0]
e = s
while not L[e].strip().startswith('s_endpgm'): e += 1
open(sys.argv[1] + '.inst', 'w').write('\n'.join(L[s:e + 1]))
lab = {}
for i in range(s, e + 1):
    m = re.match(r'^(\.LBB\S+):', L[i])
    if m: lab[m.group(1)] = i
tot = sum(1 for x in L[s:e] if x.strip().startswith('v_'))
print('instance lines', e - s, 'VALU', tot)
for i in range(s, e + 1):
    m = re.search(r'(s_branch|s_cbranch_\w+)\s+(\.LBB\S+)', L[i])
    if m and lab[m.group(2)] < i and i - lab[m.group(2)] < 1500:
        seg = L[lab[m.group(2)]:i + 1]
        nv = sum(1 for x in seg if x.strip().startswith('v_'))
        if nv >= 10:
            print(f"loop {m.group(2)} lines {lab[m.group(2)]-s}-{i-s}: VALU {nv}")
PY
