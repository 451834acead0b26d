#!/usr/bin/env python3
"""Tuning sweep for the specialised kernels (one process, interleaved variants).

For each variant (env knobs read by the library at JIT time: LONGHAIR_AMD_JIT_DEFINES,
LONGHAIR_AMD_NO_FUSED_PLAN) it times encode_batch and decode_batch on the
bench workload with HIP events and checks the bytes against the default variant.
Usage: python tools/tune.py [k m bytes stripes] > gpurun_out/tune.txt
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
import longhair_amd as lh  # noqa: E402

VARIANTS = [
    ("base", {}),
    ("noxcd", {"LONGHAIR_AMD_JIT_DEFINES": "LH_XCD=0"}),
    ("nofused", {"LONGHAIR_AMD_NO_FUSED_PLAN": "1"}),
]
KNOBS = ["LONGHAIR_AMD_JIT_DEFINES", "LONGHAIR_AMD_NO_FUSED_PLAN"]
# Large-m (windowed) variants: rows per wave and columns in flight.
VARIANTS_WIN = [
    ("base", {}),
    ("pb_branch", {"LONGHAIR_AMD_JIT_DEFINES": "LH_PB_MASK=0"}),
]


def main():
    global VARIANTS
    k, m, nbytes, stripes = (int(a) for a in sys.argv[1:5]) if len(sys.argv) >= 5 else (29, 4, 1296, 65536)
    if m > 12:
        VARIANTS = VARIANTS_WIN
    if os.environ.get("TUNE_VARIANTS"):  # name=KNOB:VALUE;KNOB:VALUE|name2=...  (JIT defines use ',')
        VARIANTS = [("base", {})]
        for item in os.environ["TUNE_VARIANTS"].split("|"):
            name, _, spec = item.partition("=")
            env = dict(kv.split(":", 1) for kv in spec.split(";") if kv)
            VARIANTS.append((name, env))
    torch.cuda.set_device(0)
    assert lh.cauchy_256_init() == 0
    X, D, rows0, _ = bench.make_workload(k, m, nbytes, stripes, seed=7)
    e = min(k, m)
    rec_view = D[:, k - e:]
    if os.environ.get("TUNE_COMPACT_REC"):  # encode into a compact [S, m, B] buffer (probe)
        rec_view = torch.empty((stripes, m, nbytes), dtype=torch.uint8, device="cuda")
    if os.environ.get("TUNE_REC_FIRST"):  # recovery blocks in slots 0..e-1 (probe)
        D = torch.roll(D, e, dims=1).contiguous()
        rows0 = torch.roll(rows0, e, dims=1).contiguous()
        rec_view = D[:, :e]
    rows = rows0.clone()
    ref_rec = None
    results = {name: ([], []) for name, _ in VARIANTS}
    reps = 3 if m > 12 else 10
    for rnd in range(int(os.environ.get('TUNE_ROUNDS', '3'))):
        for name, env in VARIANTS:
            for key in KNOBS:
                os.environ.pop(key, None)
            os.environ.update(env)
            lh.prepare(k, m, nbytes, stripes)
            lh.encode_batch(X, m, recovery=rec_view)
            torch.cuda.synchronize()
            if ref_rec is None:
                ref_rec = rec_view.clone()
            elif rnd == 0:
                assert torch.equal(rec_view, ref_rec) or "probe" in name, f"{name}: encode bytes differ"
            rows.copy_(rows0)
            if rec_view.data_ptr() != D[:, k - e:].data_ptr() and not os.environ.get("TUNE_REC_FIRST"):
                D[:, k - e:] = rec_view
            lh.decode_batch(D, rows, m)
            torch.cuda.synchronize()
            if rnd == 0:
                order = rows.long().argsort(dim=1)
                ok = torch.equal(torch.gather(D, 1, order.unsqueeze(-1).expand(-1, -1, nbytes)), X)
                assert ok or "probe" in name, f"{name}: decode did not restore the data"
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(reps):
                lh.encode_batch(X, m, recovery=rec_view)
            s1.record()
            torch.cuda.synchronize()
            results[name][0].append(s0.elapsed_time(s1) / reps)
            tot = 0.0
            for _ in range(reps):
                lh.encode_batch(X, m, recovery=rec_view)
                rows.copy_(rows0)
                d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                d0.record()
                lh.decode_batch(D, rows, m)
                d1.record()
                torch.cuda.synchronize()
                tot += d0.elapsed_time(d1)
            results[name][1].append(tot / reps)
            print(f"round {rnd} {name}: encode {results[name][0][-1]:.4f} decode {results[name][1][-1]:.4f} ms",
                  file=sys.stderr, flush=True)  # progress (a long sweep must not look hung)
    inb = k * nbytes * stripes
    print(f"k={k} m={m} bytes={nbytes} stripes={stripes} path enc={lh.batch_path(k, m, nbytes)} "
          f"dec={lh.batch_path(k, m, nbytes, True)}")
    for name, (enc, dec) in results.items():
        em, dm = min(enc), min(dec)
        print(f"{name:10s} encode {em:.4f} ms {inb / em / 1e6:8.1f} GB/s in ({(k + m) * nbytes * stripes / em / 1e6:7.1f} alg)"
              f" | decode {dm:.4f} ms {inb / dm / 1e6:8.1f} GB/s in   [enc runs {['%.3f' % x for x in enc]}]")


if __name__ == "__main__":
    main()
