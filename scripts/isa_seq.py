"""Compressed instruction sequence of one basic block of a kernel (hipcc -S output):
M = MFMA, v = VALU, L = LDS, G = vector memory load, S = store, W = s_waitcnt, n = s_nop,
s = SALU; runs collapsed (v7 = seven VALU in a row).
Usage: python scripts/isa_seq.py FILE.s KERNEL_SUBSTRING BLOCK_LABEL"""
import re
import sys

sys.path.insert(0, __file__.rsplit('/', 1)[0])
from isa_census import cat, kernel_body  # noqa: E402

CODE = {'mfma': 'M', 'valu': 'v', 'accvgpr': 'a', 'lds': 'L', 'vmem_load': 'G', 'vmem_store': 'S',
        'waitcnt': 'W', 'nop': 'n', 'salu': 's', 'branch': 'b', 'atomic': 'A'}


def main():
    f, name, label = sys.argv[1:4]
    body = kernel_body(open(f).read().splitlines(), name)
    out, inb = [], False
    for ln in body:
        s = ln.strip()
        if re.match(r'^\.LBB\S+:', s):
            inb = s.startswith(label + ':')
            continue
        if inb and s and not s.startswith(';') and not s.startswith('.'):
            out.append(CODE.get(cat(s.split()[0]), 'o'))
    seq, i = [], 0
    while i < len(out):
        j = i
        while j < len(out) and out[j] == out[i]:
            j += 1
        seq.append(out[i] + (str(j - i) if j - i > 1 else ''))
        i = j
    print(' '.join(seq))


if __name__ == '__main__':
    main()
