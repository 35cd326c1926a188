"""Instruction mix of a kernel's main loop from a hipcc --save-temps .s file:
python tools/tools_isa_loop.py file.s kernel_substring"""
import collections
import re
import sys


def loop_mix(path, sub):
    s = open(path).read()
    names = [m.group(1) for m in re.finditer(r'\n(\w+):[^\n]*@', s) if sub in m.group(1)]
    out = {}
    for name in names:
        i = s.index('\n' + name + ':')
        j = s.index('.Lfunc_end', i)
        k = s[i:j].split('\n')
        labels = {l.split(':')[0]: n for n, l in enumerate(k) if re.match(r'^\.LBB\d+_\d+:', l)}
        best = None
        for n, l in enumerate(k):
            m = re.match(r'\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
            if m and m.group(1) in labels and labels[m.group(1)] < n:
                a = labels[m.group(1)]
                body = k[a:n + 1]
                nm = sum('v_mfma' in x for x in body)
                if best is None or nm > best[0] or (nm == best[0] and n - a > best[2] - best[1]):
                    best = (nm, a, n)
        c = collections.Counter()
        for l in k[best[1]:best[2] + 1]:
            m = re.match(r'\s+([a-z_0-9]+)', l)
            if m:
                c[m.group(1)] += 1
        cls = collections.Counter()
        for op, v in c.items():
            if 'mfma' in op:
                cls['mfma'] += v
            elif op.startswith('v_'):
                cls['valu'] += v
            elif op.startswith('s_'):
                cls['salu'] += v
            elif op.startswith('ds_'):
                cls['lds'] += v
            elif op.startswith(('global_', 'buffer_')):
                cls['vmem'] += v
        out[name] = (dict(cls), sorted(((v, op) for op, v in c.items() if op.startswith('v_') and 'mfma' not in op),
                                       reverse=True)[:14])
    return out


if __name__ == "__main__":
    for n, (cls, top) in loop_mix(sys.argv[1], sys.argv[2]).items():
        print(n[:60], cls)
        print('   ', top)
