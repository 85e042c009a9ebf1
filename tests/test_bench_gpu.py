"""bench.py's multi-rank path on real hardware, on a one-GPU box: `--gpus 2` relaunches itself under
torch.distributed.run, both ranks land on cuda:0 (--share-gpus: bench_device wraps LOCAL_RANK and the
line is marked shared, n_gpus = 1 distinct device; without the flag the run exits), the gloo group
carries the barrier and the scalar max/sum of the timing rule, and rank 0 prints one JSON line
whose value is the whole-job rate (codewords of both ranks / max-over-ranks time)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_on_one_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--ncw", str(1 << 16), "--no-cpu-baseline", "--no-extras", "--share-gpus"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    ndev = torch.cuda.device_count()
    if ndev >= 2:
        assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    else:                                   # both ranks on one GPU: marked, never a scaling line
        assert line["n_gpus"] == 1 and line["ranks"] == 2 and line["shared_gpus"] is True
        assert not line["scaling"].startswith("weak")
    assert line["config"]["global_codewords"] == 2 << 16
    # value = both ranks' codewords / the max-over-ranks time
    assert abs(line["value"] - 2 * 3 * (1 << 16) * 255 / (line["ms_per_step"] * 3e-3) / 1e9) < 0.02 * line["value"]
