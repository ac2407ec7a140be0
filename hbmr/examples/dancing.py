"""Dancing links (Knuth's Algorithm X) with Sudoku and pentomino tilings, and a
distributed pentomino job (src/examples/org/apache/hadoop/examples/dancing/
{DancingLinks,Sudoku,Pentomino,DistributedPentomino}.java).

The distributed job enumerates the search tree to a fixed depth on the client,
writes one prefix per input line (NLineInputFormat, one line per map) and each
map counts the solutions below its prefix; a reducer sums them.
"""
from __future__ import annotations

import argparse
import os
import tempfile

from ..io.writable import LongWritable, Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper, Reducer
from ..mapred.formats import NLineInputFormat


class DancingLinks:
    """Exact cover over ``ncols`` columns (the first ``primary`` must be covered
    exactly once; the rest at most once).  Rows are lists of column indices."""

    def __init__(self, ncols, primary=None):
        self.ncols = ncols
        self.primary = ncols if primary is None else primary
        self.rows: list[list[int]] = []
        self.row_names: list = []

    def add_row(self, cols, name=None):
        self.rows.append(sorted(set(cols)))
        self.row_names.append(name if name is not None else len(self.rows) - 1)

    # A compact set-based Algorithm X (the column choice heuristic: fewest rows)
    def _prepare(self):
        cols = {c: set() for c in range(self.ncols)}
        for i, r in enumerate(self.rows):
            for c in r:
                cols[c].add(i)
        return cols

    @staticmethod
    def _select(cols, rows, r):
        removed = []
        for j in rows[r]:
            for i in cols[j]:
                for k in rows[i]:
                    if k != j:
                        cols[k].discard(i)
            removed.append(cols.pop(j))
        return removed

    @staticmethod
    def _deselect(cols, rows, r, removed):
        for j in reversed(rows[r]):
            cols[j] = removed.pop()
            for i in cols[j]:
                for k in rows[i]:
                    if k != j:
                        cols[k].add(i)

    def _search(self, cols, partial, on_solution, limit=None, prefix_depth=None, prefixes=None):
        primary = [c for c in cols if c < self.primary]
        if not primary:
            if prefixes is not None:
                prefixes.append(list(partial))
                return 1
            on_solution([self.row_names[r] for r in partial])
            return 1
        if prefix_depth is not None and len(partial) == prefix_depth:
            prefixes.append(list(partial))
            return 0
        c = min(primary, key=lambda x: len(cols[x]))
        count = 0
        for r in sorted(cols[c]):
            partial.append(r)
            removed = self._select(cols, self.rows, r)
            count += self._search(cols, partial, on_solution, limit, prefix_depth, prefixes)
            self._deselect(cols, self.rows, r, removed)
            partial.pop()
            if limit is not None and count >= limit:
                break
        return count

    def solve(self, on_solution=lambda s: None, limit=None, prefix=()):
        cols = self._prepare()
        for r in prefix:
            self._select(cols, self.rows, r)
        return self._search(cols, list(prefix), on_solution, limit)

    def split(self, depth):
        """All partial solutions (row index lists) of the given depth."""
        prefixes: list = []
        self._search(self._prepare(), [], lambda s: None, None, depth, prefixes)
        return prefixes


# ------------------------------------------------------------------------ Sudoku
class Sudoku:
    """9×9 (or n²×n²) Sudoku as exact cover: cell, row-digit, col-digit, box-digit."""

    def __init__(self, grid):
        self.grid = [list(r) for r in grid]
        self.n = len(grid)
        self.b = int(round(self.n ** 0.5))

    @classmethod
    def parse(cls, text):
        rows = []
        for line in text.strip().splitlines():
            toks = line.replace(",", " ").split()
            if toks:
                rows.append([0 if t in ("?", ".", "0") else int(t) for t in toks])
        return cls(rows)

    def _dlx(self):
        n, b = self.n, self.b
        dl = DancingLinks(4 * n * n)
        for r in range(n):
            for c in range(n):
                given = self.grid[r][c]
                for d in range(1, n + 1):
                    if given and d != given:
                        continue
                    box = (r // b) * b + c // b
                    dl.add_row([r * n + c, n * n + r * n + d - 1, 2 * n * n + c * n + d - 1,
                                3 * n * n + box * n + d - 1], (r, c, d))
        return dl

    def solve(self, limit=None):
        out = []

        def emit(rows):
            g = [[0] * self.n for _ in range(self.n)]
            for r, c, d in rows:
                g[r][c] = d
            out.append(g)
        self._dlx().solve(emit, limit=limit)
        return out


# ------------------------------------------------------------------------ Pentomino
_PIECES = {  # cells of each pentomino in one orientation
    "F": [(0, 1), (0, 2), (1, 0), (1, 1), (2, 1)], "I": [(0, 0), (1, 0), (2, 0), (3, 0), (4, 0)],
    "L": [(0, 0), (1, 0), (2, 0), (3, 0), (3, 1)], "N": [(0, 1), (1, 1), (2, 0), (2, 1), (3, 0)],
    "P": [(0, 0), (0, 1), (1, 0), (1, 1), (2, 0)], "T": [(0, 0), (0, 1), (0, 2), (1, 1), (2, 1)],
    "U": [(0, 0), (0, 2), (1, 0), (1, 1), (1, 2)], "V": [(0, 0), (1, 0), (2, 0), (2, 1), (2, 2)],
    "W": [(0, 0), (1, 0), (1, 1), (2, 1), (2, 2)], "X": [(0, 1), (1, 0), (1, 1), (1, 2), (2, 1)],
    "Y": [(0, 1), (1, 0), (1, 1), (2, 1), (3, 1)], "Z": [(0, 0), (0, 1), (1, 1), (2, 1), (2, 2)],
}


def _orientations(cells, fixed=False):
    outs = set()
    pts = cells
    for flip in ((False,) if fixed else (False, True)):
        p = [(r, -c) for r, c in pts] if flip else list(pts)
        for _ in range(4):
            p = [(c, -r) for r, c in p]
            mr, mc = min(r for r, _ in p), min(c for _, c in p)
            outs.add(tuple(sorted((r - mr, c - mc) for r, c in p)))
    return sorted(outs)


class Pentomino:
    """Tile a width×height board with the 12 pentominoes.  To count each
    distinct solution once, the X piece is restricted to the board's lower-left
    quadrant (removes the rotations/reflections of symmetric boards)."""

    def __init__(self, width=10, height=6):
        self.w, self.h = width, height
        names = sorted(_PIECES)
        self.names = names
        ncols = len(names) + width * height
        self.dl = DancingLinks(ncols)
        for pi, name in enumerate(names):
            for shape in _orientations(_PIECES[name]):
                ph = max(r for r, _ in shape) + 1
                pw = max(c for _, c in shape) + 1
                for y in range(height - ph + 1):
                    for x in range(width - pw + 1):
                        if name == "X" and not (x + 1 <= (width - 1) / 2 and
                                                y + 1 <= (height - 1) / 2):
                            continue
                        cells = [len(names) + (y + r) * width + (x + c) for r, c in shape]
                        self.dl.add_row([pi] + cells, (name, tuple((y + r, x + c)
                                                                  for r, c in shape)))

    def solve(self, on_solution=lambda s: None, prefix=()):
        return self.dl.solve(on_solution, prefix=prefix)

    def split(self, depth):
        return self.dl.split(depth)


# ------------------------------------------------------------------------ distributed
class PentominoMapper(Mapper):
    def configure(self, job):
        self.p = Pentomino(job.get_int("pent.width", 10), job.get_int("pent.height", 6))

    def map(self, key, value, output, reporter):
        prefix = [int(t) for t in str(value).split(",") if t]
        n = self.p.solve(prefix=prefix)
        output.collect(Text("solutions"), LongWritable(n))


class SumReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(key, LongWritable(sum(v.get() for v in values)))


def distributed_pentomino(out, width=10, height=6, depth=2, conf=None, cluster=None,
                          verbose=False):
    p = Pentomino(width, height)
    prefixes = p.split(depth)
    tmp = tempfile.mkdtemp(prefix="pent-")
    with open(os.path.join(tmp, "prefixes.txt"), "w") as f:
        for pre in prefixes:
            f.write(",".join(map(str, pre)) + "\n")
    job = JobConf(conf)
    job.set_job_name("dancingElephant")
    job.set_int("pent.width", width)
    job.set_int("pent.height", height)
    job.set_input_format(NLineInputFormat)
    job.set_int("mapred.line.input.format.linespermap", max(1, len(prefixes) // 16))
    job.set_mapper_class(PentominoMapper)
    job.set_combiner_class(SumReducer)
    job.set_reducer_class(SumReducer)
    job.set_output_key_class(Text)
    job.set_output_value_class(LongWritable)
    job.set_num_reduce_tasks(1)
    FileInputFormat.setInputPaths(job, tmp)
    FileOutputFormat.setOutputPath(job, out)
    JobClient.runJob(job, cluster=cluster, verbose=verbose)
    total = 0
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            for line in open(os.path.join(out, fn)):
                total += int(line.split("\t")[1])
    return total


def main_sudoku(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr sudoku")
    ap.add_argument("puzzle")
    a = ap.parse_args(argv)
    sols = Sudoku.parse(open(a.puzzle).read()).solve()
    for s in sols:
        print("\n".join(" ".join(map(str, r)) for r in s) + "\n")
    print(f"Found {len(sols)} solutions")
    return 0


def main_pentomino(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr pentomino")
    ap.add_argument("output")
    ap.add_argument("-width", type=int, default=10)
    ap.add_argument("-height", type=int, default=6)
    ap.add_argument("-depth", type=int, default=2)
    a = ap.parse_args(argv)
    n = distributed_pentomino(a.output, a.width, a.height, a.depth, cluster=cluster, verbose=True)
    print(f"{n} solutions")
    return 0
