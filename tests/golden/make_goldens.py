#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REAL reference.

Run in the build container only (needs /root/reference and `make -C oracle ref`):

    python tests/golden/make_goldens.py

Every expected output here is produced by the reference's own cpu_app.c
functions (oracle/_ref/ref_driver, see oracle/ref_driver.c), never by our code.
Inputs are either the reference's own data files (sort-merge-join/data/*.csv,
test/data/data_1*.csv -- committed gzip'd as fixtures) or small hand-written /
seeded CSVs written by this script.  manifest.json records, per case, the
input files, the user.h values, the joined row count and sha256 of result.csv;
small results are also committed verbatim.
"""
import gzip
import hashlib
import json
import os
import random
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")


def sha256(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def write(name, text):
    with open(os.path.join(HERE, name), "w", newline="") as f:
        f.write(text)
    return name


def gz_copy(src, name):
    with open(src, "rb") as f, gzip.GzipFile(os.path.join(HERE, name), "wb", mtime=0) as g:
        shutil.copyfileobj(f, g)
    return name


def unpack(name, tmpdir):
    """Materialise a (possibly gzip'd) fixture as a plain CSV for the driver."""
    src = os.path.join(HERE, name)
    if not name.endswith(".gz"):
        return src
    dst = os.path.join(tmpdir, name[:-3])
    with gzip.open(src, "rb") as g, open(dst, "wb") as f:
        shutil.copyfileobj(g, f)
    return dst


def run_ref(d1, d2, cfg, tmpdir, case):
    out = os.path.join(tmpdir, case + ".result.csv")
    args = [DRIVER, d1, d2, out]
    if cfg is not None:
        args += [str(x) for x in cfg]
    res = subprocess.run(args, check=True, capture_output=True, text=True)
    return out, int(res.stdout.strip().splitlines()[-1])


def table(header, rows, crlf=False):
    nl = "\r\n" if crlf else "\n"
    return nl.join([",".join(header)] + [",".join(str(v) for v in r) for r in rows]) + nl


def main():
    if not os.path.exists(DRIVER):
        sys.exit("build the reference driver first: make -C oracle ref")
    tmpdir = os.path.join(REPO, "oracle", "_ref", "golden_tmp")
    os.makedirs(tmpdir, exist_ok=True)
    cases = {}

    # --- the reference's own data files ----------------------------------
    smj = os.path.join(REF, "sort-merge-join", "data")
    tst = os.path.join(REF, "test", "data")
    gz_copy(os.path.join(smj, "data1.csv"), "data1.csv.gz")
    gz_copy(os.path.join(smj, "data2.csv"), "data2.csv.gz")
    gz_copy(os.path.join(tst, "data_1.csv"), "data_1.csv.gz")
    gz_copy(os.path.join(tst, "data_1(1).csv"), "data_1(1).csv.gz")
    specs = [
        # name, input1, input2, (c1 v1 c2 v2 k1 k2) or None for user.h defaults
        ("bundled_100k", "data1.csv.gz", "data2.csv.gz", None),
        ("test_10k", "data_1.csv.gz", "data_1(1).csv.gz", None),
        # other join / select columns on the reference data (generalised layouts)
        ("test_10k_key1_sel2", "data_1.csv.gz", "data_1(1).csv.gz", (2, 15000, 3, 1000, 1, 1)),
        ("test_10k_key3_key2", "data_1.csv.gz", "data_1(1).csv.gz", (0, 0, 0, 0, 3, 2)),
    ]

    # --- SURVEY 8(c) known-answer test ------------------------------------
    kat_r = [(7, 1, 10), (5000, 2, 20), (7, 3, 30), (9, 4, 40), (-3, 5, 50), (7, 6, 60),
             (3000000000, 7, 70), (5001, 8, 80), (5001, 9, 90)]
    kat_s = [(7, 100), (7, 200), (5001, 300), (9, 400), (3000000000, 500), (-1294967296, 600),
             (5001, 700)]
    write("kat_r.csv", table(["a", "b", "c"], kat_r))
    write("kat_s.csv", table(["x", "y"], kat_s))
    specs += [
        ("kat_all", "kat_r.csv", "kat_s.csv", (0, -5000000000, 0, -5000000000, 0, 0)),
        ("kat_sel100", "kat_r.csv", "kat_s.csv", (0, -100, 0, -100, 0, 0)),
        ("kat_default", "kat_r.csv", "kat_s.csv", None),
    ]

    # --- edge cases (seeded, small) ---------------------------------------
    rng = random.Random(20241220)
    # heavy duplicates: zip pairing + stability visible through payload columns
    dr = [(rng.randint(-5, 12), i, rng.randint(0, 99)) for i in range(400)]
    ds = [(rng.randint(-5, 12), 1000 + i) for i in range(300)]
    write("dup_r.csv", table(["k", "p", "q"], dr, crlf=True))
    write("dup_s.csv", table(["k", "p"], ds, crlf=True))
    specs += [
        ("dup_heavy", "dup_r.csv", "dup_s.csv", (0, -100, 0, -100, 0, 0)),
        ("dup_heavy_sel", "dup_r.csv", "dup_s.csv", (2, 49, 1, 1150, 0, 0)),
        ("empty_select", "dup_r.csv", "dup_s.csv", (0, 1000, 0, 1000, 0, 0)),
    ]
    # all rows share one key
    write("same_r.csv", table(["k", "p"], [(42, i) for i in range(257)]))
    write("same_s.csv", table(["k", "p"], [(42, 500 + i) for i in range(129)]))
    specs.append(("all_same_key", "same_r.csv", "same_s.csv", (0, 0, 0, 0, 0, 0)))
    # header-only table and single-row tables
    write("empty_t.csv", "k,p\n")
    write("one_r.csv", table(["k", "p"], [(77, 1)]))
    write("one_s.csv", table(["k", "p"], [(77, 2)]))
    specs += [
        ("empty_table", "empty_t.csv", "dup_s.csv", (0, -100, 0, -100, 0, 0)),
        ("single_rows", "one_r.csv", "one_s.csv", (0, 0, 0, 0, 0, 0)),
    ]
    # atoi corner cases: spaces, '+', junk suffix, 32-bit wrap, saturation,
    # CRLF, a trailing comma (extra "\n" token spills into the next row),
    # collapsed empty fields
    write("atoi_r.csv",
          "k,p,q\r\n"
          " 12,+3,-0\r\n"
          "4294967308,7abc,5\r\n"
          "99999999999999999999,1,2\r\n"
          "-2147483649,4,4\r\n"
          "12,,9,\r\n"
          "5,5,5,5\r\n"
          "8,8,8\r\n"
          "-1,\t6, 6\r\n")
    write("atoi_s.csv",
          "k,v\n"
          "12,100\n"
          "-1,200\n"
          "12,300\n"
          "2147483647,400\n"
          "-1,500\n")
    specs.append(("atoi_edge", "atoi_r.csv", "atoi_s.csv", (0, -3000000000, 0, -3000000000, 0, 0)))
    # different column counts, key not in column 0, select on a payload column
    wr = [(rng.randint(0, 50), rng.randint(-20, 20), i, rng.randint(0, 9)) for i in range(2000)]
    ws = [(i, rng.randint(0, 3), rng.randint(-20, 20), rng.randint(0, 99), 7 * i)
          for i in range(1500)]
    write("wide_r.csv", table(["a", "b", "c", "d"], wr))
    write("wide_s.csv", table(["a", "b", "c", "d", "e"], ws))
    specs.append(("wide_mixed", "wide_r.csv", "wide_s.csv", (3, 2, 3, 10, 1, 2)))
    # full int32 range random keys, partial overlap
    nr = [(rng.randint(-2**31, 2**31 - 1), i) for i in range(3000)]
    ns = [(r[0] if rng.random() < 0.4 else rng.randint(-2**31, 2**31 - 1), 10**6 + i)
          for i, r in enumerate(rng.sample(nr, 2500))]
    write("neg_r.csv", table(["k", "p"], nr))
    write("neg_s.csv", table(["k", "p"], ns))
    specs.append(("neg_wide", "neg_r.csv", "neg_s.csv", (0, -2**31 - 1, 0, -2**31 - 1, 0, 0)))

    # rows wider than 8 columns (the index-sort path; cpu_app.c's load_csv
    # takes any column count, :46-79): key and select columns not in column 0
    rng2 = random.Random(20261016)
    w12r = [[rng2.randint(-30, 30) for _ in range(12)] for _ in range(2500)]
    w12s = [[rng2.randint(-30, 30) for _ in range(12)] for _ in range(2000)]
    for i, r in enumerate(w12r):
        r[0] = i  # row ids in a payload column: stability is visible
    for i, r in enumerate(w12s):
        r[1] = 10000 + i
    write("w12_r.csv", table([f"r{c}" for c in range(12)], w12r))
    write("w12_s.csv", table([f"s{c}" for c in range(12)], w12s, crlf=True))
    w20r = [[rng2.randint(0, 999) for _ in range(20)] for _ in range(1500)]
    w20s = [[rng2.randint(0, 999) for _ in range(9)] for _ in range(1800)]
    for r in w20r:
        r[19] = rng2.randint(100, 400)
    for i, r in enumerate(w20s):
        r[0] = rng2.randint(100, 400)
        r[5] = i
    write("w20_r.csv", table([f"c{c}" for c in range(20)], w20r))
    write("w20_s.csv", table([f"d{c}" for c in range(9)], w20s))
    specs += [
        ("wide12", "w12_r.csv", "w12_s.csv", (3, -10, 11, -5, 5, 7)),
        ("wide20_9", "w20_r.csv", "w20_s.csv", (0, 300, 4, 100, 19, 0)),
        ("wide9_20", "w20_s.csv", "w20_r.csv", (4, 100, 0, 300, 0, 19)),
    ]

    for name, i1, i2, cfg in specs:
        d1, d2 = unpack(i1, tmpdir), unpack(i2, tmpdir)
        out, rows = run_ref(d1, d2, cfg, tmpdir, name)
        entry = {"inputs": [i1, i2],
                 "config": None if cfg is None else dict(zip(
                     ["SELECT_COL1", "SELECT_VAL1", "SELECT_COL2", "SELECT_VAL2",
                      "JOIN_KEY1", "JOIN_KEY2"], cfg)),
                 "rows": rows, "sha256": sha256(out), "bytes": os.path.getsize(out)}
        if os.path.getsize(out) <= 64 * 1024:
            entry["result"] = name + ".result.csv"
            shutil.copy(out, os.path.join(HERE, entry["result"]))
        cases[name] = entry
        print(f"{name:22s} rows={rows:7d} sha256={entry['sha256'][:16]}")

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_goldens.py (reference cpu_app.c via oracle/_ref)",
                   "user_h_defaults": {"SELECT_COL1": 0, "SELECT_VAL1": 5000, "SELECT_COL2": 0,
                                       "SELECT_VAL2": 5000, "JOIN_KEY1": 0, "JOIN_KEY2": 0},
                   "cases": cases}, f, indent=1, sort_keys=True)
    shutil.rmtree(tmpdir)


if __name__ == "__main__":
    main()
