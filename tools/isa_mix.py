"""Static instruction mix of kernels in a hipcc -S output: python tools/isa_mix.py file.s name_substr..."""
import sys
from collections import Counter


def bodies(path):
    cur, out = None, {}
    for line in open(path):
        if line and not line[0].isspace() and line.rstrip().endswith(':') is False and ':' in line and ' ; @' in line:
            cur = line.split(':')[0]
            out[cur] = []
            continue
        if cur and line.startswith('.Lfunc_end'):
            cur = None
        if cur and line.startswith('\t') and not line.strip().startswith(('.', ';')):
            out[cur].append(line.strip())
    return out


def mix(lines):
    c = Counter()
    for l in lines:
        op = l.split()[0]
        if 'mfma' in op:
            k = 'mfma'
        elif op.startswith('ds_read') or op.startswith('ds_load'):
            k = 'ds_read'
        elif op.startswith('ds_'):
            k = 'ds_other'
        elif op.startswith('scratch_'):
            k = 'scratch'
        elif op.startswith(('global_load', 'buffer_load')):
            k = 'vmem_ld'
        elif op.startswith(('global_', 'buffer_')):
            k = 'vmem_st'
        elif op.startswith('s_waitcnt'):
            k = 'waitcnt'
        elif op.startswith('s_'):
            k = 'salu'
        elif op.startswith('v_'):
            k = 'valu'
        else:
            k = 'other'
        c[k] += 1
    return c


if __name__ == '__main__':
    b = bodies(sys.argv[1])
    for name, lines in b.items():
        if all(s in name for s in sys.argv[2:]):
            print(name[:90], len(lines), dict(sorted(mix(lines).items())))


def blocks(lines_raw):
    """Split a kernel body (with labels) into basic blocks: [(label, [instr...])]."""
    out, cur, name = [], [], 'entry'
    for l in lines_raw:
        if l.endswith(':') and not l.startswith('\t'):
            out.append((name, cur))
            name, cur = l[:-1], []
        elif l.startswith('\t') and not l.strip().startswith(('.', ';')):
            cur.append(l.strip())
    out.append((name, cur))
    return out
