#!/usr/bin/env python3
"""Register and LDS use of a shape's specialised kernels, without a GPU: compiles the modules
(cauchy_256_jit_precompile) into a scratch cache and prints each kernel's VGPR / SGPR / spill
counts, LDS bytes and code size from the code object's metadata.

Usage: python tools/costat.py K M BYTES [enc|dec] [JIT_DEFINES]
       e.g. python tools/costat.py 29 4 1296 dec LH_DMO=1"""
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def main():
    k, m, nbytes = (int(a) for a in sys.argv[1:4])
    part = sys.argv[4] if len(sys.argv) > 4 else "dec"
    defines = sys.argv[5] if len(sys.argv) > 5 else ""
    with tempfile.TemporaryDirectory() as tmp:
        os.environ["LONGHAIR_AMD_CACHE_DIR"] = tmp
        os.environ["LONGHAIR_AMD_PRECOMPILE_PART"] = part
        if defines:
            os.environ["LONGHAIR_AMD_JIT_DEFINES"] = defines
        import longhair_amd as lh
        rc = lh.lib().cauchy_256_jit_precompile(k, m, nbytes)
        assert rc == 0, (rc, lh.last_error())
        for co in sorted(glob.glob(os.path.join(tmp, "**", "*.co"), recursive=True)):
            notes = subprocess.run([READELF, "--notes", co], capture_output=True, text=True).stdout
            for blk in re.split(r"\n\s+- \.", notes)[1:]:  # one amdhsa.kernels entry each
                mm = re.search(r"\.name:\s+(\S+)", blk)
                if not mm or mm.group(1).endswith(".kd") or "vgpr_count" not in blk:
                    continue
                name = mm.group(1)
                def f(key):
                    mm = re.search(r"\." + key + r":\s+(\d+)", blk)
                    return int(mm.group(1)) if mm else -1
                print(f"{name:28s} vgpr {f('vgpr_count'):4d} agpr {f('agpr_count'):3d} sgpr {f('sgpr_count'):3d} "
                      f"spill v/s {f('vgpr_spill_count')}/{f('sgpr_spill_count')} "
                      f"lds {f('group_segment_fixed_size'):6d}  ({os.path.getsize(co)} B object)")


if __name__ == "__main__":
    main()
