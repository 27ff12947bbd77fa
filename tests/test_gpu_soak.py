"""Short GPU soaks (tools/soak.py, tools/soak_blake3.py, tools/soak_archive.py) inside the -m gpu
suite: random shapes, erasure patterns and corrupted recovery shards through
every codec entry point on several threads with an evicting plan cache, and
random commit / damage / read / repair cases of the archive pipeline, each
checked byte for byte against oracle/ (the checker) or the original file.
The long runs are recorded in profiles/r02 (soak_r02bx/cb/cf, soak_blake3_r02ci,
soak_archive_r02by/ca/cg)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=120):
    env = dict(os.environ, **(env_extra or {}))
    p = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=timeout)
    line = next((l for l in p.stdout.splitlines() if l.startswith("{")), None)
    assert line, f"no result line (rc={p.returncode}): {p.stderr[-2000:]}"
    res = json.loads(line)
    assert p.returncode == 0 and not res["failures"], res["failures"]
    return res


@pytest.mark.parametrize("staging,slots", [("pinned", "2"), ("direct", "0")])
def test_codec_soak_short(staging, slots):
    """Both codec-object stagings; slots 0 = every object frees its slot on
    release (the empty-pool path)."""
    res = _run(["tools/soak.py", "--seconds", "6", "--threads", "4", "--seed", "7"],
               {"BFRS_PLAN_CACHE": "16", "BFRS_CODEC_STAGING": staging, "BFRS_CODEC_SLOTS": slots})
    assert res["cases"] > 100 and set(res["by_api"]) == {"host", "host_batch", "dev_batch", "objects",
                                                         "wrappers"}
    assert res["codec_staging"] == staging


def test_blake3_soak_short():
    res = _run(["tools/soak_blake3.py", "--seconds", "5", "--seed", "13"])
    assert res["messages"] > 100 and res["combines"] > 5


def test_archive_soak_short(tmp_path):
    res = _run(["tools/soak_archive.py", "--seconds", "10", "--readers", "3", "--seed", "11",
                "--workdir", str(tmp_path)])
    assert res["cases"] > 20 and res["recoverable"] > 0
