#!/usr/bin/env python3
"""Pre-populate the on-disk code-object cache (longhair_amd/jit_cache/) for the BASELINE
shapes, without a GPU, so the first GPU run does not pay the hiprtc compile (the large-m
windowed modules take minutes).  Usage: python tools/precompile.py [--all | k m bytes ...]"""
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import longhair_amd as lh  # noqa: E402

DEFAULT = [(29, 4, 1296), (128, 32, 8192), (200, 56, 65536)]
# Further shapes the GPU parity tests run through the specialised path (tests/test_gpu_parity.py).
TESTS = [(29, 2, 1296), (29, 3, 1296), (29, 8, 1296), (4, 2, 16), (10, 6, 8), (17, 6, 520), (64, 5, 4096),
         (3, 250, 24), (2, 2, 8), (29, 4, 1304), (9, 7, 72), (29, 2, 16), (10, 8, 24),
         (128, 32, 1024), (5, 3, 8), (100, 16, 2048), (40, 20, 4096), (250, 6, 2048), (10, 6, 24), (3, 2, 8),
         (64, 4, 4096), (64, 3, 4096), (64, 2, 8192), (40, 20, 6144)]
# Shapes whose pointer-table modules (cauchy_256_*_batch_ptrs, LH_PTR) the GPU tests run
# (tests/test_gpu_ptrs.py; the north-star shape is benchmarked through them too).
PTR_SHAPES = [(29, 4, 1296), (29, 8, 1296), (10, 6, 24), (64, 5, 4096), (64, 3, 4096), (40, 20, 4096),
              (128, 32, 8192), (200, 56, 65536)]
# Modules of the knob variants the GPU tests run (tests/test_gpu_parity.py KNOB_VARIANTS).
KNOB_JOBS = [((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_LDS=0,LH_PF=2,LH_NT=0,LH_XCD=0"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_LDS=0,LH_REC_FIRST=0,LH_PF_DEC=2"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_LD=2,LH_NT=0,LH_LDS_NT_DEC=0,LH_LDS_REC_FIRST=1,LH_LDS_FLAT_ST=0"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_LDG=1"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_LDG=3"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_ASM_DMA=1"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_CPS=1"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_CPS=3,LH_WPB=2,LH_WGCU=2,LH_CPS_AHEAD=1,LH_CPS_FLAT=1"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_DMO=1"}),
             ((29, 4, 1296), {"LONGHAIR_AMD_JIT_DEFINES": "LH_DMO=1,LH_DMO_AHEAD=0,LH_CPS=3"})]


def lds_sample(n, seed=606):
    """A seeded sample of n shapes served by the LDS-staged register networks:
    k in [2, 64], m in [2, 4], 16-byte-multiple blocks up to 4 KiB; encode lh_jit_encode and
    decode lh_jit_decode_fused, both staging their columns by LDS-DMA."""
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    while len(out) < n:
        k, m, b = int(rng.integers(2, 65)), int(rng.integers(2, 5)), 16 * int(rng.integers(1, 257))
        if (k, m, b) in out:
            continue
        if (lh.batch_path(k, m, b) == "jit" and lh.batch_path(k, m, b, True) == "jit-fused"
                and lh.lds_staged(k, m, b) and lh.lds_staged(k, m, b, True)):
            out.append((k, m, b))
    return out


def boundary_jobs():
    """(shape, env) of every kernel-selection boundary case in tests/test_gpu_boundaries.py
    (its own list, so the two cannot drift apart)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    import test_gpu_boundaries as tb
    jobs = [((k, m, b), dict(env)) for _, k, m, b, _, env, _, _ in tb.BOUNDARIES if "LONGHAIR_AMD_PATH" not in env]
    return jobs, tb


def sweep_shapes(tb):
    """The specialised shapes of the reference-main sweep (test_reference_main_sweep):
    every k <= 16 with 2 <= m <= 8 at the sweep's block size (small networks, seconds each)."""
    return [(k, m, 8 * (1 + (7 * k + m) % 8)) for k in range(2, 17) for m in tb._sweep_ms(k) if 2 <= m <= 8]


def main():
    if sys.argv[1:] == ["--prune"]:
        # --all, then delete the cached code objects it neither compiled nor used (outdated
        # sources, dropped shapes); the library bumps a cached object's mtime on every use.
        t0 = time.time() - 1
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--all"])
        cache = os.path.join(os.path.dirname(lh.library_path), "jit_cache")
        for f in os.listdir(cache):
            p = os.path.join(cache, f)
            if f.endswith(".co") and os.path.getmtime(p) < t0:
                os.unlink(p)
                print("pruned", f)
        return
    if sys.argv[1:2] == ["--lds-sample"]:
        # tools/stress.py --lds-sample N: the sample's encode and decode modules (and the
        # pointer-table forms of the first quarter), largest first, on every core
        n = int(sys.argv[2])
        shapes = lds_sample(n)
        jobs_list = [(sh, part, {}) for sh in shapes for part in ("enc", "dec")]
        jobs_list += [(sh, part, {"LONGHAIR_AMD_PRECOMPILE_PTR": "1"}) for sh in shapes[:n // 4] for part in ("enc", "dec")]
        jobs_list.sort(key=lambda j: -j[0][0] * j[0][2])
        cmd = [sys.executable, os.path.abspath(__file__)]

        def run1(job):
            shape, part, extra = job
            env = dict(os.environ, LONGHAIR_AMD_PRECOMPILE_PART=part, **extra)
            return subprocess.run(cmd + [str(v) for v in shape], env=env, stdout=subprocess.DEVNULL)
        with ThreadPoolExecutor(max(1, min(8, os.cpu_count() or 2))) as pool:
            runs = list(pool.map(run1, jobs_list))
        print(f"{len(shapes)} shapes, {len(jobs_list)} modules, {sum(r.returncode != 0 for r in runs)} failed")
        sys.exit(1 if any(r.returncode for r in runs) else 0)
    if sys.argv[1:] == ["--all"]:
        # One child process per (shape, part), largest network first (k * m): hiprtc is
        # single-threaded and the big modules take minutes, so the rest compile beside them
        # and none starts last.
        jobs = max(1, min(8, os.cpu_count() or 2))
        cmd = [sys.executable, os.path.abspath(__file__)]
        with ThreadPoolExecutor(jobs) as pool:
            # the BASELINE shapes with their (k, m) block-size family modules
            jobs_list = [(s, (part, {"LONGHAIR_AMD_PRECOMPILE_FAMILY": "1"})) for s in DEFAULT for part in ("enc", "dec")]
            jobs_list += [(s, None) for s in dict.fromkeys(DEFAULT + TESTS)]
            ptr_jobs = [(s, (part, {"LONGHAIR_AMD_PRECOMPILE_PTR": "1"})) for s in PTR_SHAPES for part in ("dec", "enc")]
            jobs_list += [(s, (None, env)) for s, env in KNOB_JOBS]
            # the block-size family modules the GPU tests force (tests/test_gpu_family.py)
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
            import test_gpu_family as tf
            jobs_list += [((k, m, b), ("enc", {"LONGHAIR_AMD_JIT_DEFINES": "LH_FAMILY=1"}))
                          for k, m, b, _ in tf.FAMILY_SHAPES]
            jobs_list += [((k, m, b), (part, {"LONGHAIR_AMD_JIT_DEFINES": "LH_FAMILY=1"}))
                          for k, m, b, _ in tf.FAMILY_DEC_SHAPES for part in ("dec", "enc")]
            # the families' randomised parity (test_family_random_sizes): one module per (k, m, role)
            jobs_list += [(sh, (part, {"LONGHAIR_AMD_JIT_DEFINES": "LH_FAMILY=1"}))
                          for sh in dict.fromkeys(c[:3] for c in tf.family_sample(tf.FAMILY_SAMPLE_PAIRS, sizes=1))
                          for part in ("dec", "enc")]
            jobs_list = ptr_jobs[-4:] + jobs_list + ptr_jobs[:-4]
            # kernel-selection boundaries and the reference-main sweep (test_gpu_boundaries.py)
            bj, tb = boundary_jobs()
            have = {s for s, _ in jobs_list}
            for sh, env in bj:
                if env or sh not in have:
                    jobs_list.append((sh, (None, env)))
                    have.add(sh)
            jobs_list += [(sh, None) for sh in dict.fromkeys(sweep_shapes(tb)) if sh not in have]
            have |= set(sweep_shapes(tb))
            # the specialised-kernel parity sample (test_specialised_sample), slowest first
            jobs_list += [(sh, None) for sh in sorted(tb.JIT_SAMPLE, key=lambda s: -s[0] * s[1]) if sh not in have]
            # the encode and decode modules of a shape in separate processes
            split = []
            for sh, part in jobs_list:
                p, env = part if isinstance(part, tuple) else (part, None)
                for q in ((p,) if p else ("dec", "enc")):
                    split.append((sh, (q, env) if env is not None else q))
            jobs_list = split
            jobs_list.sort(key=lambda j: -j[0][0] * j[0][1])  # (stable: parts keep their order)

            def run(job):
                shape, part = job
                env = dict(os.environ)
                if isinstance(part, tuple):
                    part, extra = part
                    env.update(extra)
                if part:
                    env["LONGHAIR_AMD_PRECOMPILE_PART"] = part
                return subprocess.run(cmd + [str(v) for v in shape], env=env)
            runs = list(pool.map(run, jobs_list))
        if any(r.returncode for r in runs):
            sys.exit(1)
        return
    else:
        args = [int(a) for a in sys.argv[1:]]
        shapes = [tuple(args[i:i + 3]) for i in range(0, len(args), 3)] or DEFAULT
    for k, m, b in shapes:
        t0 = time.time()
        rc = lh.lib().cauchy_256_jit_precompile(k, m, b)
        print(f"k={k} m={m} bytes={b}: rc={rc} {time.time() - t0:.1f} s "
              f"{lh.lib().cauchy_256_last_error().decode()}", flush=True)
        if rc != 0:
            sys.exit(1)


if __name__ == "__main__":
    main()
