#!/bin/bash
# static instruction mix of one kernel: tools/isa_count.sh FILE.hip NAME_SUBSTR [extra hipcc flags]
F=$1; K=$2; shift 2
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-gpu-rdc "$@" \
  -I$(dirname $F) --cuda-device-only -S $F -o /tmp/isa.s 2>/dev/null || exit 1
python3 - "$K" <<'PY'
import re, sys, collections
s = open('/tmp/isa.s').read(); k = sys.argv[1]
for n in re.findall(r'^(_Z\S*):', s, re.M):
    if k not in n: continue
    a = s.index(n + ':'); b = s.index('.Lfunc_end', a)
    c = collections.Counter(l.split()[0] for l in s[a:b].split('\n')
                            if l.strip() and not l.strip().startswith(('.', ';')) and not l.strip().endswith(':'))
    v = sum(x for o, x in c.items() if o.startswith('v_') and 'mfma' not in o)
    m = re.search(r'\.vgpr_count:\s+(\d+)', s[b:b+20000])
    print(n[:70], 'total', sum(c.values()), 'VALU(non-mfma)', v, 'mfma', sum(x for o, x in c.items() if 'mfma' in o))
    print('  ' + ', '.join(f'{o} {x}' for o, x in c.most_common(30)))
PY
grep -A30 "\.name: *.*$K" /tmp/isa.s | grep -E "vgpr_count|agpr_count|group_segment_fixed_size" | head -3
