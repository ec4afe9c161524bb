"""bench.py end to end on the GPU through its own entry (the driver's contract):
one JSON line from rank 0 with the per-pair check of the shard, the golden EPE and
roofline fields that are fractions of a peak (<= 1)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _fractions_are_fractions(d):
    assert 0 < d["roofline"]["frac"] <= 1.0, d["roofline"]
    assert 0 < d["path_roofline"]["frac"] <= 1.0, d["path_roofline"]
    assert 0 < d["path_roofline"]["hbm_frac"] <= d["path_roofline"]["frac"]


@pytest.mark.timeout(400)
def test_bench_c4_one_gpu_shard():
    """Config 4's per-GPU shard (8 pairs, bf16) through bench.py --gpus 1: n_gpus 1, eight
    per-pair EPEs vs the f32 HIP path, none above the reference network's own bf16 worst
    pair at this config (tests/golden/bf16_noise.json; tests/test_gpu_bf16.py)."""
    from tests.test_gpu_bf16 import _bf16_noise
    d = _bench("--gpus", "1", "--config", "c4", "--steps", "2", "--warmup", "1", "--cpu-baseline", "0",
               "--extra-configs", "")
    assert "configs" not in d
    assert d["n_gpus"] == 1 and d["config"]["global_batch"] == 8 and d["dtype"] == "bf16"
    pp = d["pair_epe_px"]["per_pair"]
    assert len(pp) == 8 and max(pp) <= max(_bf16_noise("c4")["epe_px"]), pp
    assert d["epe_px"]["per_rank"][0] < 0.25
    _fractions_are_fractions(d)


@pytest.mark.timeout(400)
def test_bench_c2_default_workload():
    """The default workload (C2 fp32, batch 1): the per-pair check against the direct-conv
    engine is at the f32 bar, and so is the golden EPE."""
    d = _bench("--gpus", "1", "--steps", "3", "--warmup", "1", "--cpu-baseline", "0", "--extra-steps", "3")
    assert d["n_gpus"] == 1 and d["config"]["global_batch"] == 1 and d["dtype"] == "f32"
    # the other single-GPU BASELINE configs ride in the same line
    assert sorted(d["configs"]) == ["c3", "c5"], d.get("configs")
    for name, dtype, batch in (("c3", "bf16", 8), ("c5", "f32", 1)):
        c = d["configs"][name]
        assert c["dtype"] == dtype and c["global_batch"] == batch and c["steps"] == 3
        assert c["value"] > 0 and abs(c["value"] - batch * 1e3 / c["ms_per_step"]) < 1e-6 * c["value"]
        assert 0 < c["roofline"]["frac"] <= 1.0 and 0 < c["path_roofline"]["frac"] <= 1.0
    assert len(d["pair_epe_px"]["per_pair"]) == 1 and d["pair_epe_px"]["max"] < 1e-3
    assert d["epe_px"]["max_over_ranks"] < 1e-3
    assert d["roofline"]["kernel"].startswith("conv3d_wino")
    _fractions_are_fractions(d)


@pytest.mark.timeout(600)
def test_bench_world2_gloo_on_one_gpu():
    """bench.py's N-rank path executed on the GPU: two ranks through the
    real launcher, gloo, both on cuda:0 -- device-side per-rank graph capture, the
    device-tensor max / gathers (host-staged for gloo), device selection.  Config 4 (bf16,
    8 pairs per rank): two per-rank step entries, 16 per-pair EPEs within the reference
    network's own bf16 worst pair, one line from rank 0.  Only RCCL itself is not exercised."""
    from tests.test_gpu_bf16 import _bf16_noise
    d = _bench("--gpus", "2", "--dist-backend", "gloo", "--config", "c4", "--steps", "2", "--warmup", "1",
               "--extra-configs", "")
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 16 and d["config"]["dist_backend"] == "gloo"
    assert [r["rank"] for r in d["per_rank_step_ms"]] == [0, 1]
    pp = d["pair_epe_px"]["per_pair"]
    assert len(pp) == 16 and max(pp) <= max(_bf16_noise("c4")["epe_px"]), pp
    assert len(d["epe_px"]["per_rank"]) == 2
    # rank r's pairs come from the rank-seeded stream: the two shards are different inputs
    assert pp[:8] != pp[8:]
    assert "cpu_baseline" not in d
    _fractions_are_fractions(d)
