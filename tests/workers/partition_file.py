"""Worker: auto-partition result written to ``partition_file`` and reused with
``load_partition`` (argv: save|load|api path); ``api`` hands the saved assignment to
``DistributedModel.load_partition`` instead of the config key."""
import json
import sys

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp


def main():
    mode, path = sys.argv[1], sys.argv[2]
    cfg = {"pipeline_parallel_degree": 2, "microbatches": 2, "auto_partition": True, "partition_file": path}
    if mode == "load":
        cfg["load_partition"] = True
    smp.init(cfg)
    torch.manual_seed(0)
    net = nn.Sequential(*[nn.Sequential(nn.Linear(32, 32), nn.Tanh()) for _ in range(6)])
    model = smp.DistributedModel(net)
    mm = smp.state.module_manager
    assert mm.partition_loaded == (mode == "load")
    if mode == "api":
        with open(path) as f:
            model.load_partition(json.load(f)["partition"])
        assert mm.partition_loaded
    assert model.get_module_for_param(net[3][0].weight) is net[3][0]

    @smp.step
    def train(model, x):
        out = model(x).sum()
        model.backward(out)
        return out

    train(model, torch.randn(8, 32))
    parts = mm.partition_dict()
    assert set(parts.values()) == {0, 1}, parts
    if mode in ("load", "api"):
        with open(path) as f:
            saved = json.load(f)["partition"]
        assert parts == saved, (parts, saved)
    print(f"rank {smp.rank()} OK {mode}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
