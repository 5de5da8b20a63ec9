"""Instruction census of one kernel in a hipcc -S assembly file (CPU-side, no GPU).

Usage: python scripts/isa_census.py FILE.s KERNEL_SUBSTRING [--gaps] [--blocks]

Prints per-category counts over the kernel body, and with --gaps the histogram of vector
instructions (VALU, excluding MFMA) issued between consecutive MFMAs inside each basic
block -- the placement the one-wave-per-SIMD schedule depends on (MI355X_MICROARCH.md:
<= 5 single-issue fillers hide per v_mfma_f32_32x32x16_bf16 gap).  --blocks lists the basic
blocks with their MFMA / VALU counts (the tile loop is the block with the most MFMAs)."""
import collections
import re
import sys


def kernel_body(lines, name):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r'^_Z\S*' + re.escape(name) + r'\S*:\s*(;.*)?$', l) and name in l:
            start = i
        elif start is not None and (l.startswith('.Lfunc_end') or l.strip().startswith('.size')):
            return lines[start:i]
    raise SystemExit(f'kernel {name} not found')


def cat(op):
    if 'mfma' in op:
        return 'mfma'
    if op.startswith('v_accvgpr'):
        return 'accvgpr'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_waitcnt'):
        return 'waitcnt'
    if op.startswith('s_nop'):
        return 'nop'
    if op.startswith('s_cbranch') or op.startswith('s_branch'):
        return 'branch'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_load', 'buffer_load', 'flat_load')):
        return 'vmem_load'
    if op.startswith(('global_store', 'buffer_store', 'flat_store')):
        return 'vmem_store'
    if op.startswith(('global_atomic', 'buffer_atomic', 'flat_atomic')):
        return 'atomic'
    return 'other'


def main():
    f, name = sys.argv[1], sys.argv[2]
    lines = open(f).read().splitlines()
    body = kernel_body(lines, name)
    counts = collections.Counter()
    blocks = []  # (label, [ops])
    cur = ['entry', []]
    for l in body:
        s = l.strip()
        if not s or s.startswith(';') or s.startswith('.'):
            if re.match(r'^\.LBB\S+:', s):
                blocks.append(cur)
                cur = [s.rstrip(':'), []]
            continue
        if s.endswith(':'):
            continue
        op = s.split()[0]
        counts[cat(op)] += 1
        cur[1].append(op)
    blocks.append(cur)
    print('kernel', name, 'instructions', sum(counts.values()))
    for k, v in counts.most_common():
        print(f'  {k:10s} {v}')
    if '--blocks' in sys.argv:
        for lab, ops in blocks:
            c = collections.Counter(cat(o) for o in ops)
            if c['mfma'] or len(ops) > 40:
                print(f'{lab:12s} n={len(ops):5d} mfma={c["mfma"]:4d} valu={c["valu"]:5d} lds={c["lds"]:3d} '
                      f'vmem={c["vmem_load"]:3d} wait={c["waitcnt"]:3d} nop={c["nop"]:3d} salu={c["salu"]:3d}')
    if '--gaps' in sys.argv:
        hist = collections.Counter()
        lead = tail = 0
        for lab, ops in blocks:
            seen = False
            n = 0
            for o in ops:
                c = cat(o)
                if c == 'mfma':
                    if seen:
                        hist[min(n, 40)] += 1
                    else:
                        lead += n
                    seen = True
                    n = 0
                elif c in ('valu', 'accvgpr'):
                    n += 1
            if seen:
                tail += n
        print('VALU between consecutive MFMAs (gap -> count):')
        print('  ', dict(sorted(hist.items())))
        print('  VALU before the first / after the last MFMA of their blocks:', lead, tail)


if __name__ == '__main__':
    main()
