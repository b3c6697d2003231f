"""Run-length view of one kernel's instruction stream in a hipcc -S listing (labels kept):
python tools/asm_runs.py file.s name_substring [first_line last_line]"""
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
i = next(k for k in range(len(s)) if False) if False else None
import re
m = next(m for m in re.finditer(r'^(_Z\S+):\s*;', s, re.M) if pat in m.group(1))
i = m.end()
j = s.index('.Lfunc_end', i)
CL = ['v_mfma', 'scratch_', 'v_accvgpr_read', 'v_accvgpr_write', 'v_accvgpr_mov', 'ds_read_b128', 'ds_read_b64_tr', 'ds_read',
      'ds_write', 'v_exp', 's_waitcnt', 'v_cvt_pk', 'global_load', 's_barrier', 'v_cndmask', 'v_cmp', 's_cbranch', 'buffer_',
      'global_store', 's_setprio', 's_nop']
out, prev, cnt = [], None, 0
for l in s[i:j].split('\n'):
    l = l.strip()
    if not l or l.startswith(';') or (l.startswith('.') and not l.startswith('.LBB')):
        continue
    if l.startswith('.LBB'):
        if prev:
            out.append(f'{prev}x{cnt}')
        out.append('\n' + l.split()[0])
        prev, cnt = None, 0
        continue
    op = l.split()[0]
    c = next((k for k in CL if op.startswith(k)), 'valu' if op.startswith('v_') else ('salu' if op.startswith('s_') else op))
    if c == prev:
        cnt += 1
    else:
        if prev:
            out.append(f'{prev}x{cnt}')
        prev, cnt = c, 1
out.append(f'{prev}x{cnt}')
print(' '.join(out))
