"""Go ``text/tabwriter`` emulation (AlignLeft, minwidth 0, padchar ' ').

``kubectl-inspect-gpushare`` formats its tables with ``tabwriter.NewWriter(os.Stdout, 0, 0,
2, ' ', 0)`` (``cmd/inspect/display.go:16,142``). To stay output-compatible the column
algorithm is reproduced: a column block is a run of consecutive lines that have a
tab-terminated cell in that column; its width is the widest cell + padding; the text after
a line's last tab is not part of any column.
"""
from __future__ import annotations


def format_tabs(text: str, padding: int = 2) -> str:
    lines = [ln.split("\t") for ln in text.split("\n")]
    widths: dict[tuple[int, int], int] = {}

    def fmt(line0: int, line1: int, col: int):
        i = line0
        while i < line1:
            if len(lines[i]) - 1 <= col:
                i += 1
                continue
            j, w = i, 0
            while j < line1 and len(lines[j]) - 1 > col:
                w = max(w, len(lines[j][col]) + padding)
                j += 1
            for k in range(i, j):
                widths[(k, col)] = w
            fmt(i, j, col + 1)
            i = j

    fmt(0, len(lines), 0)
    out = []
    for li, cells in enumerate(lines):
        parts = [c.ljust(widths[(li, ci)]) for ci, c in enumerate(cells[:-1])]
        parts.append(cells[-1])
        out.append("".join(parts))
    return "\n".join(out)


class TabWriter:
    def __init__(self, padding: int = 2):
        self.buf: list[str] = []
        self.padding = padding

    def write(self, s: str):
        self.buf.append(s)

    def flush(self) -> str:
        return format_tabs("".join(self.buf), self.padding)
