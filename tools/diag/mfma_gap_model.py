"""Static issue model of an MFMA-paced loop: for each gap between consecutive v_mfma in a kernel's
hot loop, the vector/scalar issue cycles of what sits in the gap (MI355X_MICROARCH.md issue-cost
row: transcendental 8, other VALU 4, s_nop N -> N+1, an MFMA holds issue for 8 of its 32
cycles), and the gap's time = max(32, 8 + issue). Prints the per-gap table and the loop total.
    python tools/diag/mfma_gap_model.py file.s KERNEL_SUBSTRING"""
import re
import sys

TRANS = ('v_exp_', 'v_log_', 'v_rcp_', 'v_rsq_', 'v_sqrt_', 'v_sin_', 'v_cos_')


def cost(op, line):
    if op.startswith('s_nop'):
        return int(line.split()[1]) + 1
    if op.startswith(TRANS):
        return 8
    if op.startswith(('v_', 'ds_', 'buffer_', 'global_', 'scratch_')):
        return 4
    if op.startswith('s_'):
        return 1
    return 0


def main():
    s = open(sys.argv[1]).read()
    m = re.search(r'^(_Z\w*' + re.escape(sys.argv[2]) + r'\w*):', s, re.M)
    end = s.find('.Lfunc_end', m.end())
    body = [l.strip() for l in s[m.end():end].split('\n')]
    hdr = [i for i, l in enumerate(body) if 'Loop Header' in l and l.startswith('.LBB')][0]
    lab = body[hdr].split(':')[0]
    back = max(i for i, l in enumerate(body) if re.search(r's_(cbranch_\w+|branch) ' + re.escape(lab) + r'\b', l))
    seg = [l for l in body[hdr:back + 1] if l and not l.startswith(';') and not l.endswith(':')]
    gaps, cur, waits = [], 0, []
    pre = 0
    first = True
    for l in seg:
        op = l.split()[0]
        if op.startswith('v_mfma'):
            if first:
                pre, first = cur, False
            else:
                gaps.append(cur)
            cur = 0
            continue
        cur += cost(op, l)
    tail = cur
    t = sum(max(32, 8 + g) for g in gaps)
    over = sum(max(0, 8 + g - 32) for g in gaps)
    print(f'MFMAs {len(gaps) + 1}  issue before first {pre}  after last {tail}')
    print(f'gap model: {t} cycles for {len(gaps)} gaps (MFMA floor {32 * len(gaps)}), overflow {over}')
    print('gaps over 24 issue cycles:', [(i, g) for i, g in enumerate(gaps) if g > 24])


if __name__ == '__main__':
    main()
