"""bench.py rank launch: `--gpus N` without WORLD_SIZE starts N ranks itself
through torch.distributed.run; a WORLD_SIZE that disagrees with --gpus is refused.  CPU only
(`--launch-check`: the ranks join a gloo group and report, no GPU is touched)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(kw)
    return e


def test_self_launch_starts_n_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=REPO,
                       env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout
    d = json.loads(line[0])
    assert d["world"] == 2 and d["n_gpus"] == 2
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1]
    assert sorted(x["local"] for x in d["ranks"]) == [0, 1]
    assert len({x["pid"] for x in d["ranks"]}) == 2


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--launch-check"], cwd=REPO,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_strong_scaling_launch_shards_eight_sequences():
    """BASELINE configs[3] launch (--sequences-total 8 --gpus N): every rank owns its contiguous
    block of the 8 sequences (ssf.dist.sequence_shard), together exactly the 8."""
    for n in (2, 3):
        r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--sequences-total", "8",
                            "--launch-check"], cwd=REPO, env=_env(), capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        ranks = sorted(d["ranks"], key=lambda x: x["rank"])
        assert [s for x in ranks for s in x["shard"]] == list(range(8))
        assert max(len(x["shard"]) for x in ranks) - min(len(x["shard"]) for x in ranks) <= 1
