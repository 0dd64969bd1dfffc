"""Joint placement of the pending queue: exact bin-packing of pods onto GPU HBM.

Online best fit (the gpushare extender's policy, one pod at a time) strands HBM whenever the
node's mixed pod sizes do not arrive in a convenient order: at 8 MI355X with BASELINE config 3's
32 pods it packs 30-31 of them in random or size-sorted order (``bench.py`` ``fill_orders``),
though all 32 fit. The extender sees the whole queue of unscheduled ``aliyun.com/gpu-mem``
pods, so it can place them jointly: ``pack`` assigns items to bins maximising the number of
pods placed, then the HBM placed — a depth-first search over items in decreasing size with
best-fit as the starting incumbent, bins with equal free space tried once per level, and a
bound on what the remaining items could still add. The search stops after ``budget`` node
expansions and keeps the best assignment found (never worse than best fit).
"""
from __future__ import annotations


def best_fit(free: list[int], sizes: list[int], order: list[int]) -> list[int | None]:
    left = list(free)
    out: list[int | None] = [None] * len(sizes)
    for k in order:
        fits = [b for b, f in enumerate(left) if f >= sizes[k]]
        if fits:
            b = min(fits, key=lambda b: (left[b] - sizes[k], b))
            out[k] = b
            left[b] -= sizes[k]
    return out


def _score(assign: list[int | None], sizes: list[int]) -> tuple[int, int]:
    return sum(1 for a in assign if a is not None), sum(s for a, s in zip(assign, sizes) if a is not None)


def pack(free: list[int], sizes: list[int], budget: int = 200_000) -> list[int | None]:
    """Bin index per item (None = not placed) maximising (items placed, size placed)."""
    n = len(sizes)
    if n == 0:
        return []
    order = sorted(range(n), key=lambda k: -sizes[k])
    # incumbent: the better of best fit in arrival order (what the online extender would do)
    # and in decreasing size order
    best = max((best_fit(free, sizes, list(range(n))), best_fit(free, sizes, order)),
               key=lambda a: _score(a, sizes))
    best_score = _score(best, sizes)
    if best_score[0] == n:
        return best
    suffix_cnt = [0] * (n + 1)
    suffix_sz = [0] * (n + 1)
    for i in range(n - 1, -1, -1):
        suffix_cnt[i] = suffix_cnt[i + 1] + 1
        suffix_sz[i] = suffix_sz[i + 1] + sizes[order[i]]
    left = list(free)
    cur: list[int | None] = [None] * n
    expansions = 0

    def dfs(i: int, cnt: int, sz: int, skipped: int) -> bool:
        """``skipped``: size of the last item left out — equal items are interchangeable, so
        once one of a size is left out the rest of that size are too (no symmetric branches)."""
        nonlocal best, best_score, expansions
        expansions += 1
        if (cnt, sz) > best_score:
            best, best_score = list(cur), (cnt, sz)
            if cnt == n:
                return True
        if i == n or expansions > budget:
            return False
        room = sum(left)
        if (cnt + suffix_cnt[i], sz + min(suffix_sz[i], room)) <= best_score:
            return False
        k = order[i]
        s = sizes[k]
        if s != skipped:
            tried = set()
            for b in sorted(range(len(left)), key=lambda b: (left[b] - s, b)):
                f = left[b]
                if f < s or f in tried:
                    continue
                tried.add(f)
                left[b] -= s
                cur[k] = b
                if dfs(i + 1, cnt + 1, sz + s, 0):
                    return True
                left[b] += s
                cur[k] = None
        return dfs(i + 1, cnt, sz, s)        # leave this one out

    dfs(0, 0, 0, 0)
    return best
