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


def test_live_pmc_parsing(tmp_path):
    """roofline.traffic from rocprofv3 --pmc CSVs: only the named kernel's
    launches, averaged; FETCH_SIZE doubled (gfx950), both in KiB."""
    sys.path.insert(0, REPO)
    import bench

    kernel = "haar_strip_kernel<5, 3, unsigned char, false>"
    for counter, vals in (("FETCH_SIZE", (100.0, 300.0)), ("WRITE_SIZE", (7.0, 9.0))):
        d = tmp_path / counter / "host" / "123"
        d.mkdir(parents=True)
        rows = ["Kernel_Name,Counter_Name,Counter_Value"]
        rows += [f'"void wicca::{kernel}(wicca::LLParams)",{counter},{v}' for v in vals]
        rows.append(f'"wicca::synth_u8_kernel(unsigned char*)",{counter},999999')
        rows.append(f'"void wicca::{kernel}(wicca::LLParams)",OTHER,5')
        (d / "123_counter_collection.csv").write_text("\n".join(rows) + "\n")
    fetch = bench.pmc_counter_kib(str(tmp_path / "FETCH_SIZE"), "FETCH_SIZE", kernel)
    write = bench.pmc_counter_kib(str(tmp_path / "WRITE_SIZE"), "WRITE_SIZE", kernel)
    assert (fetch, write) == (200.0, 8.0)
    assert bench.pmc_counter_kib(str(tmp_path / "FETCH_SIZE"), "FETCH_SIZE", "nope") is None
    hbm = bench.pmc_hbm_bytes(fetch, write)
    assert hbm == {"read_bytes": 409600.0, "write_bytes": 8192.0, "hbm_bytes_per_launch": 417792.0}
