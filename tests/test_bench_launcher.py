"""bench.py ``--gpus N`` on CPU (no GPU): the launcher starts N rank processes, forwards only
rank 0's JSON line, reports ``n_gpus == N``, and fails when a rank fails.  The rank body is a
fake (no torch / GPU): it goes through ``bench.main`` under the launcher's environment, so the
WORLD_SIZE check and the result line are the real ones."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

# A rank: records its environment in a file, then prints bench.result_line on rank 0
# (FAKE_FAIL_RANK makes that rank exit 3 instead; FAKE_HANG_RANK makes it sleep).
FAKE_RANK = r"""
import json, os, sys, time
sys.path.insert(0, {root!r})
import bench
def fake_run_rank(args):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    with open(os.path.join({tmp!r}, f"rank{{rank}}.json"), "w") as f:
        json.dump({{k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                              "MASTER_PORT")}} | {{"gpus": args.gpus}}, f)
    if os.environ.get("FAKE_FAIL_RANK") == str(rank):
        sys.exit(3)
    if os.environ.get("FAKE_HANG_RANK") == str(rank):
        time.sleep(600)
    print(f"rank {{rank}} chatter")          # stdout of every rank; only rank 0's is forwarded
    if rank == 0:
        cfg = bench.CONFIGS[args.config]
        print(json.dumps(bench.result_line(args, cfg, world, 0.1, [0.1] * args.runs)), flush=True)
bench.run_rank = fake_run_rank
sys.exit(bench.main(sys.argv[1:]))
"""


def _worker(tmp_path, argv):
    return [sys.executable, "-c", FAKE_RANK.format(root=ROOT, tmp=str(tmp_path)), *argv]


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_starts_n_ranks_and_forwards_rank0_line(tmp_path, capfd, n):
    argv = ["--gpus", str(n), "--steps", "20", "--warmup", "5"]
    rc = bench.launch_workers(argv, n, worker=_worker(tmp_path, argv))
    assert rc == 0
    out = capfd.readouterr().out
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 2 and lines[0] == "rank 0 chatter"          # rank 0 only
    line = json.loads(lines[1])
    assert line["n_gpus"] == n
    assert line["config"]["global_batch"] == 256 * n
    assert line["config"]["parallelism"] == f"dp{n}"
    assert line["value"] == pytest.approx(200.0)          # optimizer steps/s, not n x
    assert line["samples_per_s"] == pytest.approx(200.0 * 256 * n)
    assert line["batch_gradients_per_s"] == pytest.approx(200.0 * n)
    assert line["runs"] == [200.0] * 5
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(n)]
    assert [e["RANK"] for e in envs] == [str(r) for r in range(n)]
    assert [e["LOCAL_RANK"] for e in envs] == [str(r) for r in range(n)]
    assert {e["WORLD_SIZE"] for e in envs} == {str(n)}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert {e["gpus"] for e in envs} == {n}


def test_launcher_fails_when_a_rank_fails(tmp_path, monkeypatch):
    argv = ["--gpus", "3", "--steps", "20"]
    monkeypatch.setenv("FAKE_FAIL_RANK", "2")
    assert bench.launch_workers(argv, 3, worker=_worker(tmp_path, argv)) == 3


def test_launcher_stops_the_other_ranks_after_a_failure(tmp_path, monkeypatch):
    argv = ["--gpus", "2", "--steps", "20"]
    monkeypatch.setenv("FAKE_FAIL_RANK", "1")
    monkeypatch.setenv("FAKE_HANG_RANK", "0")        # rank 0 would wait forever in a collective
    t0 = time.time()
    assert bench.launch_workers(argv, 2, worker=_worker(tmp_path, argv), grace_s=2.0) == 3
    assert time.time() - t0 < 60


def test_external_launcher_world_size_must_match_gpus(tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run(_worker(tmp_path, ["--gpus", "4"]), env=env, capture_output=True, text=True)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    assert not (tmp_path / "rank0.json").exists()


def test_external_launcher_takes_world_size_when_gpus_is_omitted(tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="1")
    r = subprocess.run(_worker(tmp_path, ["--steps", "20"]), env=env, capture_output=True, text=True)
    assert r.returncode == 0
    assert json.load(open(tmp_path / "rank1.json"))["gpus"] == 2


def test_single_gpu_runs_in_process(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    code = FAKE_RANK.format(root=ROOT, tmp=str(tmp_path)).replace(
        'rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])',
        'rank, world = 0, 1; os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", '
        'MASTER_ADDR="-", MASTER_PORT="-")')
    r = subprocess.run([sys.executable, "-c", code, "--steps", "20"], env=env, capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.splitlines()[-1])
    assert line["n_gpus"] == 1 and line["config"]["parallelism"] == "single"
    assert json.load(open(tmp_path / "rank0.json"))["gpus"] == 1


def test_pendulum_config_flops_match_survey():
    assert bench.step_flops(bench.CONFIGS["pendulum"]) / 1e9 == pytest.approx(1.710, rel=1e-3)
