#!/usr/bin/env python3
"""Where the time of a one-stripe drop-in call forced onto the GPU goes (round-2 verdict:
the GPU drop-in decode took 59 us against 35 us for the encode).  Runs CALLS encode and
decode calls of k29/m4/1296 with host pointers under LONGHAIR_AMD_DISPATCH=gpu and prints
the per-call wall time; run it under `rocprofv3 --kernel-trace --memory-copy-trace --stats`
to split each call into copies and kernels.  Usage: dropin_probe.py [CALLS]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (adds tests/ to sys.path)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    import lhutil
    import longhair_amd as lh
    k, m, nbytes = 29, 4, 1296
    lib = lh.lib()
    prev = lh.set_dispatch("gpu")
    d0 = lhutil.fill(7, k * nbytes)
    out = bench.per_call_us(lib.cauchy_256_encode, lib.cauchy_256_decode, k, m, nbytes, calls, d0,
                            bench.dropin_blocks(k, m, nbytes, d0))
    out["launches_last_decode"] = lh.last_launch()
    lh.set_dispatch(prev)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
