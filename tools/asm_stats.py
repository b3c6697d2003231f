"""Instruction statistics of one kernel in a hipcc -S listing: python tools/asm_stats.py file.s substring"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
for m in re.finditer(r'^(_Z\S+):\s*;', s, re.M):
    n = m.group(1)
    if pat not in n:
        continue
    i = m.end()
    j = s.index('.Lfunc_end', i)
    body = s[i:j]
    keys = ['scratch_store', 'scratch_load', 'v_mfma', 'v_accvgpr_write', 'v_accvgpr_read', 'ds_read', 'ds_write',
            'global_load', 's_waitcnt', 'v_exp', 's_barrier', 'v_mov_b32', 's_cbranch']
    print(n[:90], 'lines', body.count('\n'), ' '.join(f'{k}={body.count(k)}' for k in keys))
