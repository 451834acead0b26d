"""The block-size families without a GPU (jit.cpp jit_family_ok, jit_codec.hip LH_FAMILY): for
the encode and for the fused decode, hiprtc compiles one code object for k29/m4 that serves
1 296, 1 312 and 2 592-byte blocks, and the shapes outside the family keep
their size-keyed modules."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _precompile(tmp, env_extra, shapes, part):
    env = dict(os.environ, LONGHAIR_AMD_CACHE_DIR=str(tmp), LONGHAIR_AMD_PRECOMPILE_PART=part, **env_extra)
    args = [str(v) for sh in shapes for v in sh]
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "precompile.py")] + args, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return sorted(f for f in os.listdir(tmp) if f.endswith(".co"))


@pytest.mark.parametrize("part", ["enc", "dec"])
def test_one_family_module_serves_three_block_sizes(tmp_path, part):
    import longhair_amd as lh
    what = 8 if part == "enc" else 9
    env = {"LONGHAIR_AMD_JIT_DEFINES": "LH_FAMILY=1"}
    os.environ.update(env)
    try:
        assert [lh.lib().cauchy_256_batch_path(29, 4, b, what) for b in (1296, 1312, 2592)] == [1, 1, 1]
        # outside the family: not a 16-byte multiple; more than 64 lanes; m > 6
        assert [lh.lib().cauchy_256_batch_path(*sh, what) for sh in ((29, 4, 1304), (29, 4, 4112), (29, 7, 1296))] == [0, 0, 0]
        if part == "dec":  # e_max > 4; more than 8 Block.row bytes per lane (3 lanes for k = 29)
            assert [lh.lib().cauchy_256_batch_path(*sh, 9) for sh in ((29, 5, 1296), (29, 4, 192))] == [0, 0]
    finally:
        for key in env:
            os.environ.pop(key, None)
    cos = _precompile(tmp_path, env, [(29, 4, 1296), (29, 4, 1312), (29, 4, 2592)], part)
    assert len(cos) == 1, cos
