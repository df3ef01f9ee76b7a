"""Sharded-data-parallel (ZeRO-3 style) configuration.

The reference builds a DeepSpeed stage-3 config from defaults + ``sdp_*`` keys + an
optional JSON file and validates it (`smp/backend/zero_config.py:13-131`,
`ds_config_defaults.json:1-31`).  DeepSpeed is not part of this framework: the same
dictionary drives our native sharded-DP engine (`parallel/sharded_dp.py`), so we keep
the key names users know, and the same validation rules:

* stage must be 3; ``contiguous_gradients`` and ``cpu_offload`` must be off;
* the shard degree cannot exceed the data-parallel degree;
* fp16 in the JSON requires fp16 in the smp config;
* hierarchical all-gather is only meaningful when a shard spans more than one node.
"""
import collections.abc
import copy
import json

from .exceptions import SMPInvalidArgumentError

_DEFAULTS = {
    "train_batch_size": 1,
    "train_micro_batch_size_per_gpu": 1,
    "prescale_gradients": False,
    "zero_optimization": {
        "stage": 3,
        "overlap_comm": True,
        "contiguous_gradients": False,
        "reduce_bucket_size": 5e8,
        "stage3_param_persistence_threshold": 1e6,
        "stage3_max_reuse_distance": 1e9,
        "stage3_max_live_parameters": 1e9,
        "stage3_prefetch_bucket_size": 5e8,
        "zero2d_shard_size": 1,
        "zero2d_hierarchy_allgather": True,
        "cpu_offload": False,
        "reduce_scatter": True,
    },
    "gradient_clipping": 1.0,
}


def _merge(base, override):
    for k, v in override.items():
        if isinstance(v, collections.abc.Mapping):
            base[k] = _merge(dict(base.get(k, {})), v)
        else:
            base[k] = v
    return base


def construct_zero2d_config_dict(cfg, core):
    if not cfg.zero2d_enabled():
        return {}
    conf = copy.deepcopy(_DEFAULTS)
    z = conf["zero_optimization"]
    z["zero2d_shard_size"] = cfg.sharded_data_parallel_degree
    z["reduce_bucket_size"] = cfg.sdp_reduce_bucket_size
    z["stage3_param_persistence_threshold"] = cfg.sdp_param_persistence_threshold
    z["stage3_max_live_parameters"] = cfg.sdp_max_live_parameters
    z["zero2d_hierarchy_allgather"] = cfg.sdp_hierarchical_allgather
    conf["gradient_clipping"] = cfg.sdp_gradient_clipping
    conf["train_batch_size"] = core.dp_size()
    if cfg.fp16:
        conf["fp16"] = {"enabled": True, "loss_scale": 0, "initial_scale_power": 20, "loss_scale_window": 1000}
    if cfg.bf16:
        conf["bf16"] = {"enabled": True}
    if cfg._sharded_data_parallelism_config is not None:
        with open(cfg._sharded_data_parallelism_config, "r", encoding="utf-8") as f:
            conf = _merge(conf, json.load(f))
    validate_zero2d_config(conf, cfg, core)
    return conf


def validate_zero2d_config(conf, cfg, core):
    z = conf["zero_optimization"]
    if z.get("contiguous_gradients"):
        raise SMPInvalidArgumentError("contiguous_gradients must be false for sharded data parallelism.")
    if z.get("cpu_offload"):
        raise SMPInvalidArgumentError("cpu_offload must be false for sharded data parallelism.")
    if z.get("stage") != 3:
        raise SMPInvalidArgumentError("Only stage 3 is supported in sharded data parallelism.")
    shard = z["zero2d_shard_size"]
    if shard > core.dp_size():
        raise SMPInvalidArgumentError(
            f"Sharding degree ({shard}) cannot be larger than the data parallelism degree ({core.dp_size()})."
        )
    if not cfg.fp16 and conf.get("fp16", {}).get("enabled", False):
        raise SMPInvalidArgumentError("fp16 in the sharded-DP config requires fp16 in the smp config.")
    if shard <= core.local_size():
        z["zero2d_hierarchy_allgather"] = False
