#!/usr/bin/env python3
"""Export the reference's Cauchy generator constants as a raw binary blob.

The generator rows of the code are *data*: CAUCHY_MATRIX_2..6 (hand-improved rows for
m = 2..6) and the X/Y vectors used to rebuild rows for m >= 7
(/root/reference/cauchy_tables_256.inc:63-564).  They were produced offline by a
search (docs/tabgen.cpp) and cannot be regenerated here, yet every encoded byte depends
on them.  This script parses the .inc text once, in the build container, and writes the
byte values (no source text) to longhair_amd/data/cauchy_tables_256.bin:

    offset     size   content
    0          254    M2  (1 x 254, stride 254)   cauchy_tables_256.inc:63
    254        506    M3  (2 x 253, stride 253)   :78
    760        756    M4  (3 x 252, stride 252)   :107
    1516       1004   M5  (4 x 251, stride 251)   :150
    2520       1250   M6  (5 x 250, stride 250)   :207
    3770       256    Y[256]                      :290
    4026       30876  X[30876]                    :315
    total      34902

Usage: python tools/extract_tables.py [/root/reference/cauchy_tables_256.inc] [out.bin]
"""
import hashlib
import re
import sys

ORDER = [("CAUCHY_MATRIX_2", 254), ("CAUCHY_MATRIX_3", 506), ("CAUCHY_MATRIX_4", 756),
         ("CAUCHY_MATRIX_5", 1004), ("CAUCHY_MATRIX_6", 1250), ("CAUCHY_MATRIX_Y", 256),
         ("CAUCHY_MATRIX_X", 30876)]


def parse(text):
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    arrays = {}
    for m in re.finditer(r"(CAUCHY_MATRIX_\w+)\s*\[([^\]]*)\]\s*=\s*\{(.*?)\}", text, flags=re.S):
        declared = eval(m.group(2), {"__builtins__": {}})  # e.g. "3 * 252"
        vals = [int(v) for v in m.group(3).replace("\n", " ").split(",") if v.strip()]
        assert len(vals) <= declared
        # C zero-fills a shorter initializer (Y[] lists 254 of its 256 entries).
        arrays[m.group(1)] = vals + [0] * (declared - len(vals))
    return arrays


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/cauchy_tables_256.inc"
    out = sys.argv[2] if len(sys.argv) > 2 else "longhair_amd/data/cauchy_tables_256.bin"
    arrays = parse(open(src).read())
    blob = bytearray()
    for name, size in ORDER:
        vals = arrays[name]
        assert len(vals) == size, (name, len(vals), size)
        assert all(0 <= v < 256 for v in vals)
        blob += bytes(vals)
    open(out, "wb").write(blob)
    print(out, len(blob), hashlib.sha256(blob).hexdigest())


if __name__ == "__main__":
    main()
