"""bench.py --gpus N launches its own N rank processes (no external torchrun): each child gets torchrun's
environment. CPU-only: the children here are a tiny script that records its environment."""
import json
import os
import sys
import tempfile

import bench


def test_launcher_sets_rank_environment():
    with tempfile.TemporaryDirectory() as d:
        child = os.path.join(d, "child.py")
        with open(child, "w") as f:
            f.write("import json, os, sys\n"
                    "keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT']\n"
                    "json.dump({k: os.environ.get(k) for k in keys}, open(os.path.join(sys.argv[1], "
                    "'rank%s.json' % os.environ['RANK']), 'w'))\n")
        rc = bench.launch_ranks(4, [sys.executable, child, d])
        assert rc == 0
        envs = [json.load(open(os.path.join(d, f"rank{r}.json"))) for r in range(4)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_launcher_propagates_failure():
    rc = bench.launch_ranks(2, [sys.executable, "-c",
                                "import os, sys, time; r = int(os.environ['RANK']); time.sleep(0.1); sys.exit(3 if r == 1 else 0)"])
    assert rc == 3


def test_c3_config_matches_reference_quick_experiment():
    c = bench.CONFIGS["c3"]
    assert c["batch"] == 512 and c["cls"] == "DisentangledConditionalVAE"
    assert c["opt"]["type"] == "adam" and c["opt"]["lr"] == 5e-4 and c["clip"] == 0.5
    assert c["kwargs"]["hidden_channels"] == 32 and tuple(c["kwargs"]["ch_mult"]) == (1, 2, 4)
    assert c["kwargs"]["dropout"] == 0.1 and c["loss"]["type"] == "disentangled_vae"
