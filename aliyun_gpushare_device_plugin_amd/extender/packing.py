"""Joint placement of the pending queue: exact bin-packing of pods onto GPU HBM.

Online best fit (the gpushare extender's policy, one pod at a time) strands HBM whenever the
node's mixed pod sizes do not arrive in a convenient order: at 8 MI355X with BASELINE config 3's
32 pods it packs 30-31 of them in random or size-sorted order (``bench.py`` ``fill_orders``),
though all 32 fit. The extender sees the whole queue of unscheduled ``aliyun.com/gpu-mem``
pods, so it can place them jointly: ``pack`` assigns items to bins maximising the number of
pods placed, then the HBM placed — a depth-first search over items in decreasing size with
best-fit as the starting incumbent, bins with equal free space tried once per level, an exact
fit taken without alternatives, and a bound on what the remaining items could still add (free
space smaller than the smallest item is waste; items larger than every free space are out). The search stops after ``budget`` node
expansions (or ``deadline_s``) and keeps the best assignment found (never worse than best fit).

Scale: bins are kept as buckets of equal free space (a heap of bin indices per value, the
values sorted), so best fit is O(log) per item and the search branches over *distinct* free
values — a cluster's thousands of GPUs have a few hundred distinct free amounts at most. The
exact search runs for queues and bin sets up to ``EXACT_MAX_ITEMS`` / ``EXACT_MAX_VALUES``;
beyond that the better best fit (arrival order or decreasing size) is the plan.
"""
from __future__ import annotations

import bisect
import time

EXACT_MAX_ITEMS = 160        # the search recurses once per item
EXACT_MAX_VALUES = 320       # distinct free amounts it branches over
PLACE_ALL_MAX_BINS = 128     # bin completion recurses once per bin


class _Buckets:
    """Bins grouped by free space: value -> sorted bin indices, plus the sorted values."""

    def __init__(self, free: list[int]):
        self.by: dict[int, list[int]] = {}
        for b, f in enumerate(free):
            self.by.setdefault(f, []).append(b)      # appended in index order: already sorted
        self.keys = sorted(self.by)

    def take(self, f: int, b: int | None = None) -> int:
        """Remove bin ``b`` (default: the lowest-index one) from the bins with free space ``f``."""
        lst = self.by[f]
        b = lst.pop(0) if b is None else lst.pop(bisect.bisect_left(lst, b))
        if not lst:
            del self.by[f]
            self.keys.pop(bisect.bisect_left(self.keys, f))
        return b

    def put(self, f: int, b: int) -> None:
        lst = self.by.get(f)
        if lst is None:
            self.by[f] = [b]
            bisect.insort(self.keys, f)
        else:
            bisect.insort(lst, b)

    def best(self, s: int) -> int | None:
        """The smallest free value that holds ``s`` (best fit), or None."""
        i = bisect.bisect_left(self.keys, s)
        return self.keys[i] if i < len(self.keys) else None


def best_fit(free: list[int], sizes: list[int], order: list[int]) -> list[int | None]:
    """Each item in ``order`` to the bin it fills most tightly (lowest index on ties)."""
    bk = _Buckets(free)
    out: list[int | None] = [None] * len(sizes)
    for k in order:
        f = bk.best(sizes[k])
        if f is not None:
            b = bk.take(f)
            out[k] = b
            bk.put(f - sizes[k], b)
    return out


def _score(assign: list[int | None], sizes: list[int]) -> tuple[int, int]:
    return sum(1 for a in assign if a is not None), sum(s for a, s in zip(assign, sizes) if a is not None)


class _Budget(Exception):
    pass


def place_all(free: list[int], sizes: list[int], budget: int = 200_000) -> list[int] | None:
    """A bin per item with every item placed, or None (none exists, or the budget ran out).

    Bin completion (Korf's algorithm, for bins of different sizes): bins are filled one at a
    time, smallest first, each with a *maximal* subset of the remaining items (one no remaining
    item could still join: a non-maximal fill is never better). The total space the bins may
    leave empty is the slack, free space minus item size, so with little slack — the hard
    case for item-by-item search, a node whose pods exactly fill its GPUs — only fills that
    waste almost nothing are tried. Subsets are enumerated over items in decreasing size,
    fuller fills first, and equal sizes are tried once per level; when the bins left all have
    the same size, the largest item left goes into the current one."""
    n = len(sizes)
    slack = sum(free) - sum(sizes)
    if n == 0:
        return []
    if slack < 0:
        return None
    order = sorted(range(n), key=lambda k: -sizes[k])
    bins = sorted(range(len(free)), key=lambda b: (free[b], b))
    assign: list[int | None] = [None] * n
    steps = 0

    def fill(bi: int, left_items: list[int], waste_left: int) -> bool:
        if not left_items:
            return True
        if bi == len(bins) or sizes[left_items[0]] > max(free[b] for b in bins[bi:]):
            return False
        cap = free[bins[bi]]
        lo = cap - waste_left                 # this bin must hold at least this much
        chosen: list[int] = []

        def sub(j0: int, total: int) -> bool:
            nonlocal steps
            steps += 1
            if steps > budget:
                raise _Budget
            tried = set()
            for j in range(j0, len(left_items)):
                k = left_items[j]
                sz = sizes[k]
                if total + sz > cap or sz in tried:
                    continue
                tried.add(sz)
                chosen.append(k)
                if sub(j + 1, total + sz):
                    return True
                chosen.pop()
            if total < lo:
                return False
            cs = set(chosen)
            rest = [k for k in left_items if k not in cs]
            if rest and sizes[rest[-1]] <= cap - total:
                return False                  # not maximal: the smallest remaining item still fits
            for k in chosen:
                assign[k] = bins[bi]
            if fill(bi + 1, rest, waste_left - (cap - total)):
                return True
            for k in chosen:
                assign[k] = None
            return False

        if all(free[b] == cap for b in bins[bi:]):
            # the remaining bins are interchangeable: the largest remaining item may as well be
            # in this one (removes the bin-order symmetry)
            chosen.append(left_items[0])
            return sub(1, sizes[left_items[0]])
        return sub(0, 0)

    try:
        ok = fill(0, order, slack)
    except _Budget:
        return None
    return [a for a in assign] if ok else None   # type: ignore[misc]


def pack(free: list[int], sizes: list[int], budget: int = 200_000,
         deadline_s: float | None = None) -> list[int | None]:
    """Bin index per item (None = not placed) maximising (items placed, size placed)."""
    n = len(sizes)
    if n == 0:
        return []
    if not free:
        return [None] * n
    order = sorted(range(n), key=lambda k: -sizes[k])
    # incumbent: the better of best fit in arrival order (what the online extender would do)
    # and in decreasing size order
    best = max((best_fit(free, sizes, list(range(n))), best_fit(free, sizes, order)),
               key=lambda a: _score(a, sizes))
    best_score = _score(best, sizes)
    if best_score[0] == n or n > EXACT_MAX_ITEMS or len(set(free)) > EXACT_MAX_VALUES:
        return best
    if sum(sizes) <= sum(free) and len(free) <= PLACE_ALL_MAX_BINS:
        full = place_all(free, sizes, budget // 2)
        if full is not None:
            return full
    desc = [sizes[k] for k in order]                 # sizes in search order (non-increasing)
    neg = [-x for x in desc]                         # ascending, for bisect
    suffix_sz = [0] * (n + 1)
    for i in range(n - 1, -1, -1):
        suffix_sz[i] = suffix_sz[i + 1] + desc[i]
    bk = _Buckets(free)
    smallest = desc[-1]
    cur: list[int | None] = [None] * n
    expansions = 0
    stop_at = None if deadline_s is None else time.monotonic() + deadline_s

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
        if stop_at is not None and not expansions & 255 and time.monotonic() > stop_at:
            expansions = budget + 1
            return False
        # bound: space in a bin smaller than the smallest remaining item is wasted, and items
        # larger than the largest free space cannot be placed any more
        keys = bk.keys
        if not keys:
            return False
        lo = bisect.bisect_left(keys, smallest)
        usable = sum(f * len(bk.by[f]) for f in keys[lo:])
        big = keys[-1]
        first_fit = max(i, bisect.bisect_left(neg, -big))   # items i.. before this are > big
        fit_cnt = n - first_fit
        if (cnt + fit_cnt, sz + min(suffix_sz[i], usable)) <= best_score:
            return False
        s = desc[i]
        k = order[i]
        if s != skipped:
            j = bisect.bisect_left(keys, s)
            # best fit first; an item that exactly fills a bin goes there: any solution placing
            # it elsewhere can swap it with that bin's remaining contents
            cands = list(keys[j:j + 1]) if j < len(keys) and keys[j] == s else list(keys[j:])
            for f in cands:
                b = bk.take(f)
                bk.put(f - s, b)
                cur[k] = b
                if dfs(i + 1, cnt + 1, sz + s, 0):
                    return True
                bk.take(f - s, b)
                bk.put(f, b)
                cur[k] = None
        return dfs(i + 1, cnt, sz, s)        # leave this one out

    dfs(0, 0, 0, 0)
    return best
