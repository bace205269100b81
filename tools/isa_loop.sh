# Dump a kernel's innermost-loop ISA and register use: tools/isa_loop.sh <kernel-substring> [label]
set -e
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -o /tmp/isa/kernels.s \
  "$(dirname "$0")/../plate_inverse_problem_amd/csrc/kernels.hip" 2>/dev/null
python3 - "$1" <<'PY'
import re, sys, collections
s = open('/tmp/isa/kernels.s').read().split('\n')
pat = sys.argv[1]
starts = [i for i, l in enumerate(s) if re.match(r'^_ZN3pfr\S*:', l) and pat in l]
for st in starts:
    en = next(i for i in range(st, len(s)) if s[i].startswith('.Lfunc_end'))
    body = [l for l in s[st:en] if l.strip() and not l.strip().startswith(';')]
    name = s[st][:70]
    meta = '\n'.join(s[en:en + 400])
    vg = re.search(re.escape(s[st][:-1].split(':')[0]) + r'\.num_vgpr, (\d+)', meta)
    print(name, 'vgpr', vg.group(1) if vg else '?')
    # innermost loops: label ... backward branch to it
    labels = {l.split(':')[0]: k for k, l in enumerate(body) if re.match(r'^\.LBB\S+:', l)}
    for k, l in enumerate(body):
        m = re.match(r'\s*s_cbranch_\w+\s+(\.LBB\S+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            seg = body[labels[m.group(1)]:k + 1]
            c = collections.Counter(x.split()[0] for x in seg if not x.startswith('.'))
            print('  loop', m.group(1), 'len', len(seg), {kk: v for kk, v in c.items() if 'load' in kk or 'waitcnt' in kk or 'fma' in kk or 'mul' in kk})
PY
