"""bench.py's multi-rank harness on CPU: `bench.py --gpus 2` started directly relaunches itself as
two ranks through torch.distributed.run (127.0.0.1 rendezvous, gloo), keeps the barrier +
max-over-ranks timing, and rank 0 prints ONE JSON line with n_gpus == 2."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_launches_two_ranks():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--harness-check", "--steps", "3", "--warmup", "1", "--ncw", "4096"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["config"]["codewords_total"] == 2 * 4096
    assert rec["config"]["parallelism"] == "shard2"
