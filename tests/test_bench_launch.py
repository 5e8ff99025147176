"""CPU: ``bench.py --gpus N`` starts N ranks by itself.

The parent starts ``torch.distributed.run`` as a child (it never touches the
GPU and never execs); a WORLD_SIZE that disagrees with --gpus is refused.
``--dry-run`` stops every rank before any torch / HIP call.
"""
import json
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


@pytest.mark.parametrize("n", [3, 8])  # 8: BASELINE configs[3], 1024 x 8K over 8 GPUs
def test_gpus_n_spawns_n_ranks(n):
    out = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], env=_env(),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr
    # ranks share the pipe: take every JSON object, whatever the line breaks
    lines = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", out.stdout)]
    assert sorted(d["rank"] for d in lines) == list(range(n))
    assert sorted(d["local_rank"] for d in lines) == list(range(n))
    assert all(d["world"] == n for d in lines)


def test_world_size_mismatch_refused():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"],
                         env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                         capture_output=True, text=True, timeout=60)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr


def test_default_is_one_rank():
    out = subprocess.run([sys.executable, BENCH, "--dry-run"], env=_env(),
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert json.loads(out.stdout.strip()) == {"rank": 0, "local_rank": 0, "world": 1}
