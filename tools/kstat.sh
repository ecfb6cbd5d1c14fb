#!/bin/bash
# usage: kstat.sh <build_dir> [kernel]
O=$(readlink -f $1)/ppo_ffn.hip.o
K=${2:-_Z12k_update_ffnILi2ELi9ELi2ELb0EEv11UpdateBatch}
cd /tmp
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=/tmp/fb_$$.bin $O
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/fb_$$.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/co_$$.co
/opt/rocm/lib/llvm/bin/llvm-objdump -d --symbolize-operands /tmp/co_$$.co > /tmp/s_$$.s
awk "/$K>:/{f=1;next} /^[0-9a-f]+ <_Z/{if(f)exit} f" /tmp/s_$$.s > /tmp/k_$$.s
/opt/rocm/lib/llvm/bin/llvm-readelf --notes /tmp/co_$$.co 2>/dev/null | grep -A40 "$K" | grep -E "\.vgpr_count|\.agpr_count|\.sgpr_spill|\.vgpr_spill|\.sgpr_count" | head -5
python3 - /tmp/k_$$.s <<'PY'
import re, collections, sys
lines = open(sys.argv[1]).read().split('\n')
lab = {}
for idx, l in enumerate(lines):
    m = re.match(r'^[0-9a-f]+ <(L\d+)>:', l.strip())
    if m: lab[m.group(1)] = idx
loops = []
for idx, l in enumerate(lines):
    m = re.search(r's_(cbranch_\w+|branch)\s+(L\d+)', l)
    if m and m.group(2) in lab and lab[m.group(2)] < idx:
        loops.append((idx - lab[m.group(2)], lab[m.group(2)], idx, m.group(2)))
loops.sort(reverse=True)
print('kernel instrs', sum(1 for l in lines if re.match(r'^\s+[a-z]', l)))
for L in loops[:5]:
    seg = lines[L[1]:L[2]+1]
    ins = [re.match(r'^\s+([a-z_0-9]+)', s) for s in seg]
    c = collections.Counter(x.group(1) for x in ins if x)
    print("loop", L[1], L[2], "len", sum(c.values()), 'mfma', c['v_mfma_f32_16x16x4_f32'], 'accr', c['v_accvgpr_read_b32'], 'accw', c['v_accvgpr_write_b32'], 'readlane', c['v_readlane_b32'], 'valu', sum(v for k,v in c.items() if k.startswith('v_')), 's_nop', c['s_nop'], 'salu', sum(v for k,v in c.items() if k.startswith('s_')), 'dpp', sum(v for k,v in c.items() if 'dpp' in k), 'cnd', c['v_cndmask_b32_e64']+c['v_cndmask_b32_e32'], 'ds', sum(v for k,v in c.items() if k.startswith('ds_')))
PY
rm -f /tmp/fb_$$.bin /tmp/co_$$.co /tmp/s_$$.s /tmp/k_$$.s
