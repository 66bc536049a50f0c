"""Regenerate tests/golden/ (run in the build container, where /root/reference
exists):

    make -C oracle ref && python tests/golden/make_golden.py

* mtx/      the reference's own loader fixtures (ReadMatrixMarket/matrices/
            {b1_ss,bcspwr01,one}.mtx, copied as data) plus edge-case files
            written by this script (symmetric / pattern / integer / complex /
            0-based / unsorted+duplicates / skew / empty rows / rectangular /
            malformed);
* ref_csr/  what the REFERENCE loader (oracle/_ref/ref_dump, compiled from
            /root/reference/ReadMatrixMarket sources) returns for each file at
            outputBase 0/1 and transpose 0/1 — the loader parity vectors;
* kat.json  known-answer values recorded in SURVEY §0.7 / §8c (MKL probes).
"""
from __future__ import annotations

import json
import os
import random
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_MTX = "/root/reference/ReadMatrixMarket/matrices"
REF_DUMP = os.path.join(ROOT, "oracle", "_ref", "ref_dump")
MTX = os.path.join(HERE, "mtx")
OUT = os.path.join(HERE, "ref_csr")

HDR = "%%MatrixMarket matrix coordinate {field} {sym}\n"


def write(name: str, text: str) -> None:
    with open(os.path.join(MTX, name), "w") as f:
        f.write(text)


def entries(lines):
    return "".join(f"{e}\n" for e in lines)


def edge_cases() -> list[str]:
    rnd = random.Random(1234)
    files = []

    # symmetric real, lower triangle stored, shuffled order
    lower = [(i, j) for i in range(1, 9) for j in range(1, i + 1) if (i * 7 + j * 3) % 4 != 1 or i == j]
    rnd.shuffle(lower)
    write("sym_lower.mtx", HDR.format(field="real", sym="symmetric") + "% lower stored\n"
          + f"8 8 {len(lower)}\n" + entries(f"{i} {j} {rnd.uniform(-2, 2):.17g}" for i, j in lower))
    files.append("sym_lower.mtx")

    # symmetric with upper-triangle storage (mirror goes to the lower side)
    upper = [(j, i) for i, j in lower]
    write("sym_upper.mtx", HDR.format(field="real", sym="symmetric")
          + f"8 8 {len(upper)}\n" + entries(f"{i} {j} {0.5 + i - j * 0.25:.6f}" for i, j in upper))
    files.append("sym_upper.mtx")

    # symmetric with some pairs stored twice ((i,j) and (j,i)): mirror skips them
    both = [(1, 1), (2, 1), (1, 2), (3, 3), (3, 1), (4, 2), (2, 4), (4, 4), (2, 2), (5, 5), (5, 3)]
    write("sym_both.mtx", HDR.format(field="real", sym="symmetric")
          + f"5 5 {len(both)}\n" + entries(f"{i} {j} {i * 10 + j}" for i, j in both))
    files.append("sym_both.mtx")

    # pattern general
    pat = sorted({(rnd.randint(1, 12), rnd.randint(1, 12)) for _ in range(40)})
    write("pattern_general.mtx", HDR.format(field="pattern", sym="general")
          + f"12 12 {len(pat)}\n" + entries(f"{i} {j}" for i, j in pat))
    files.append("pattern_general.mtx")

    # pattern symmetric (like bcspwr01)
    ps = sorted({(max(a, b), min(a, b)) for a, b in ((rnd.randint(1, 10), rnd.randint(1, 10)) for _ in range(25))})
    ps += [(i, i) for i in range(1, 11) if (i, i) not in ps]
    write("pattern_sym.mtx", HDR.format(field="pattern", sym="symmetric")
          + f"10 10 {len(ps)}\n" + entries(f"{i} {j}" for i, j in ps))
    files.append("pattern_sym.mtx")

    # integer symmetric (values via %lld)
    isym = [(i, j) for i in range(1, 7) for j in range(1, i + 1) if (i + j) % 2 == 0]
    write("integer_sym.mtx", HDR.format(field="integer", sym="symmetric")
          + f"6 6 {len(isym)}\n" + entries(f"{i} {j} {i * 100 - j * 7}" for i, j in isym))
    files.append("integer_sym.mtx")

    # complex general: real part only
    cg = [(1, 1), (2, 1), (2, 2), (3, 2), (3, 3), (1, 3)]
    write("complex_general.mtx", HDR.format(field="complex", sym="general")
          + f"3 3 {len(cg)}\n" + entries(f"{i} {j} {i + 0.25 * j} {-j}" for i, j in cg))
    files.append("complex_general.mtx")

    # 0-based general file (auto-detected, loadMatrixMarket.cpp:135,144-154)
    zb = [(0, 0), (1, 0), (1, 1), (2, 2), (3, 1), (3, 3), (0, 3), (2, 0)]
    write("zero_based.mtx", HDR.format(field="real", sym="general")
          + f"4 4 {len(zb)}\n" + entries(f"{i} {j} {1.5 * (i + 1) - j}" for i, j in zb))
    files.append("zero_based.mtx")

    # unsorted entries with duplicate coordinates (pins the qsort order)
    dup = []
    for _ in range(120):
        i, j = rnd.randint(1, 9), rnd.randint(1, 9)
        dup.append((i, j, rnd.randint(-50, 50) / 8.0))
    for _ in range(30):
        i, j, _v = rnd.choice(dup)
        dup.append((i, j, rnd.randint(-50, 50) / 8.0))
    rnd.shuffle(dup)
    write("unsorted_dups.mtx", HDR.format(field="real", sym="general")
          + f"9 9 {len(dup)}\n" + entries(f"{i} {j} {v}" for i, j, v in dup))
    files.append("unsorted_dups.mtx")

    # skew-symmetric: the loader treats it as general (only 'S' mirrors)
    sk = [(2, 1), (3, 1), (3, 2), (4, 3), (1, 1)]
    write("skew.mtx", HDR.format(field="real", sym="skew-symmetric")
          + f"4 4 {len(sk)}\n" + entries(f"{i} {j} {i - j + 0.5}" for i, j in sk))
    files.append("skew.mtx")

    # empty rows (rows 2, 5, 6 empty), enough entries that count >= m+1
    er = [(1, 1), (1, 3), (1, 7), (3, 2), (3, 3), (4, 4), (4, 1), (7, 7), (7, 1), (8, 8), (8, 2)]
    write("empty_rows.mtx", HDR.format(field="real", sym="general")
          + f"8 8 {len(er)}\n" + entries(f"{i} {j} {0.1 * i + j}" for i, j in er))
    files.append("empty_rows.mtx")

    # rectangular 4 x 6 general
    rc = [(1, 6), (1, 1), (2, 5), (3, 3), (4, 2), (4, 6), (2, 2), (3, 4)]
    write("rect.mtx", HDR.format(field="real", sym="general")
          + f"4 6 {len(rc)}\n" + entries(f"{i} {j} {i * j}" for i, j in rc))
    files.append("rect.mtx")

    # comment lines, upper-case banner words, tabs and a blank line before the size line
    write("comments_ws.mtx", "%%MatrixMarket MATRIX Coordinate REAL General\n% c1\n%c2\n\n"
          "3 3 4\n1\t1\t1.0e0\n  2 2   -2.5\n3 3 3.25e-1\n3\t1\t7\n")
    files.append("comments_ws.mtx")

    # a moderately sized random general matrix (scientific notation, denormals)
    big = sorted({(rnd.randint(1, 300), rnd.randint(1, 300)) for _ in range(2500)})
    vals = [rnd.choice([rnd.uniform(-1e3, 1e3), rnd.uniform(-1e-310, 1e-310), 1e-40, -3.5e38])
            for _ in big]
    write("random_300.mtx", HDR.format(field="real", sym="general")
          + f"300 300 {len(big)}\n" + entries(f"{i} {j} {v:.17e}" for (i, j), v in zip(big, vals)))
    files.append("random_300.mtx")

    # malformed inputs: every one must fail (ok = 0) in both loaders
    write("bad_banner.mtx", "%MatrixMarket matrix coordinate real general\n2 2 1\n1 1 1\n")
    write("array.mtx", "%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
    write("nnz_mismatch.mtx", HDR.format(field="real", sym="general") + "3 3 4\n1 1 1\n2 2 2\n3 3 3\n")
    write("out_of_range.mtx", HDR.format(field="real", sym="general") + "3 3 2\n1 1 1\n4 2 2\n")
    write("bad_type.mtx", "%%MatrixMarket matrix coordinate quaternion general\n2 2 1\n1 1 1\n")
    files += ["bad_banner.mtx", "array.mtx", "nnz_mismatch.mtx", "out_of_range.mtx", "bad_type.mtx"]
    return files


def main() -> int:
    if not os.path.exists(REF_DUMP):
        print("oracle/_ref/ref_dump missing: run `make -C oracle ref` first", file=sys.stderr)
        return 1
    os.makedirs(MTX, exist_ok=True)
    os.makedirs(OUT, exist_ok=True)
    files = []
    for f in ("b1_ss.mtx", "bcspwr01.mtx", "one.mtx"):
        shutil.copyfile(os.path.join(REF_MTX, f), os.path.join(MTX, f))
        files.append(f)
    files += edge_cases()
    manifest = []
    for f in files:
        for base in (0, 1):
            for tr in (0, 1):
                out = os.path.join(OUT, f"{f[:-4]}_b{base}_t{tr}.bin")
                subprocess.run([REF_DUMP, os.path.join(MTX, f), str(base), str(tr), out],
                               check=True, capture_output=True)
                manifest.append({"file": f, "base": base, "transpose": tr,
                                 "dump": os.path.relpath(out, HERE)})
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1)
    kat = {
        "source": "SURVEY.md §0.7 and §8c (probes of MKL 2021.4 LAPACKE_dlarnv / dcsrilu0 / "
                  "mkl_sparse_d_trsv against the reference fixtures)",
        "dlarnv1_seed0001_first3": [0.12062469795087694, 0.6438459108216854, 0.06234171577016312],
        "dlarnv2_seed0001_first3": [-0.75875060409824613, 0.28769182164337082, -0.87531656845967376],
        "bcspwr01": {"A.nnz": 131, "rowptr_m": 85, "upper_entries": 0,
                     "ilu_LLt_solve_x1_first4": [31, -28, 23, -23], "ilu_LLt_solve_x1_maxabs": 48},
        "b1_ss": {"structural_zero": 0, "row0": [[1, 1.0], [2, 1.0], [3, 1.0]],
                  "row1": [[1, -1.0], [4, 0.45]]},
        "one": {"spmv_is_identity": True, "ilu_solve_x1": 1.0},
    }
    with open(os.path.join(HERE, "kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1)
    print(f"wrote {len(manifest)} reference dumps for {len(files)} files")
    return 0


if __name__ == "__main__":
    sys.exit(main())
