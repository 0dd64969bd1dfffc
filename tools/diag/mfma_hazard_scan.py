"""Scan a kernel's .s for inline-asm MFMA results read or overwritten by another instruction
before the MFMA has retired (the compiler does not pad around asm). For every v_mfma, its vdst
register range is followed until enough issue cycles have passed (an MFMA ~ 8 cycles of issue,
s_nop N ~ N+1, other instructions 4), and any non-MFMA instruction touching the range is printed.
    python tools/diag/mfma_hazard_scan.py file.s KERNEL_SUBSTRING [cycles]"""
import re
import sys


def regs(tok):
    m = re.match(r'([va])\[(\d+):(\d+)\]', tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r'([va])(\d+)$', tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def main():
    path, name = sys.argv[1], sys.argv[2]
    need = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    s = open(path).read()
    m = re.search(r'^(_Z\w*' + re.escape(name) + r'\w*):', s, re.M)
    end = s.find('.Lfunc_end', m.end())
    body = [l.strip() for l in s[m.end():end].split('\n')]
    body = [l for l in body if l and not l.startswith(';') and not l.startswith('.') and not l.endswith(':')]
    bad = 0
    for i, l in enumerate(body):
        if not l.startswith('v_mfma'):
            continue
        dst = regs(l.split()[1].rstrip(','))
        cyc = 0
        for k in range(i + 1, len(body)):
            x = body[k]
            op = x.split()[0]
            if op.startswith('s_nop'):
                cyc += int(x.split()[1]) + 1
            elif op.startswith('v_mfma'):
                cyc += 8
                # a chained MFMA taking the whole tuple as C is handled by the hardware
                ops = [t.rstrip(',') for t in x.split()[1:]]
                if regs(ops[0]) == dst and regs(ops[-1]) == dst:
                    continue
                touched = set().union(*[regs(t) for t in ops]) if ops else set()
                if touched & dst:
                    print(f'{i}: {l}\n   -> {k}: {x}  (after ~{cyc} cycles)')
                    bad += 1
            elif op.startswith('s_branch') or op.startswith('s_cbranch') or op.startswith('s_setpc'):
                cyc += 4
            else:
                cyc += 4
                touched = set()
                for t in re.split(r'[\s,]+', x)[1:]:
                    touched |= regs(t)
                if touched & dst:
                    print(f'{i}: {l}\n   -> {k}: {x}  (after ~{cyc} cycles)')
                    bad += 1
                    break
            if cyc >= need:
                break
    print('hazards:', bad)


if __name__ == '__main__':
    main()
