"""Schema-driven configuration.

Behavioural parity with the reference engine (`smp/backend/config.py:42-305`):
types, choices, bounds, formula defaults (``pipeline_parallel_degree + 2``), cross-key
``needs``/``needs_not``/``needs_any`` checks that only apply to non-default values,
dependency-ordered resolution, aliases, rejection of unknown keys, deprecation warnings,
``SM_HP_MP_PARAMETERS`` JSON overrides and the two post-constraints (non-interleaved
pipeline with ``active_microbatches != microbatches`` becomes interleaved; attention
checkpointing is disabled under PP>1).

Implementation is our own: formulas are parsed with :mod:`ast` and evaluated over the
already-resolved values, and resolution is a topological sort of the ``after`` graph.
"""
import ast
import json
import operator
import os

import yaml

from .exceptions import SMPUnsupportedError, SMPConfigError, SMPConfigTypeError, SMPInvalidArgumentError
from .logger import get_logger

logger = get_logger()

_SCHEMA_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config.yaml")
_TYPES = {"int": int, "float": float, "bool": bool, "str": str, "none": type(None), None: type(None)}
_BINOPS = {
    ast.Add: operator.add,
    ast.Sub: operator.sub,
    ast.Mult: operator.mul,
    ast.Div: operator.truediv,
    ast.FloorDiv: operator.floordiv,
}


def load_schema():
    with open(_SCHEMA_PATH, "r") as f:
        return yaml.safe_load(f)


def _eval_formula(expr, values):
    """Evaluate ``"{a} + 2"``-style expressions. Non-string values pass through."""
    if not isinstance(expr, str) or "{" not in expr:
        return expr
    src = expr.replace("{", "").replace("}", "")
    tree = ast.parse(src, mode="eval")

    def ev(node):
        if isinstance(node, ast.Expression):
            return ev(node.body)
        if isinstance(node, ast.Constant):
            return node.value
        if isinstance(node, ast.Name):
            if node.id not in values:
                raise SMPConfigError(f"formula {expr!r} references unresolved key {node.id}")
            return values[node.id]
        if isinstance(node, ast.BinOp) and type(node.op) in _BINOPS:
            return _BINOPS[type(node.op)](ev(node.left), ev(node.right))
        if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
            return -ev(node.operand)
        raise SMPConfigError(f"unsupported formula {expr!r}")

    out = ev(tree)
    if isinstance(out, float) and out.is_integer():
        out = int(out)
    return out


def _resolution_order(schema):
    order, done, visiting = [], set(), set()

    def visit(k):
        if k in done:
            return
        if k in visiting:
            raise SMPConfigError(f"cyclic config dependency at {k}")
        visiting.add(k)
        for d in schema[k].get("after", []) or []:
            visit(d)
        visiting.discard(k)
        done.add(k)
        order.append(k)

    for k in schema:
        visit(k)
    return order


class ModelParallelConfig:
    """Validated configuration. Every schema key becomes an attribute."""

    def __init__(self, config=None):
        config = dict(config or {})
        env = os.environ.get("SM_HP_MP_PARAMETERS")
        if env:
            config.update(json.loads(env))

        schema = load_schema()
        self._schema = schema

        # aliases
        for key, spec in schema.items():
            alias = spec.get("alias")
            if alias and alias in config:
                if key in config and config[key] != config[alias]:
                    raise SMPInvalidArgumentError(
                        f"Conflicting values {config[key]} and {config[alias]} for {key} and its alias {alias}."
                    )
                config[key] = config.pop(alias)

        unknown = [k for k in config if k not in schema]
        if unknown:
            raise SMPInvalidArgumentError(f"Unrecognized config parameter {unknown[0]}.")

        values = {}
        for key in _resolution_order(schema):
            spec = schema[key]
            if key in config:
                values[key] = self._validate(key, spec, config[key], values)
            else:
                values[key] = self._default(spec, values)

        self._values = values
        self._input_config = config
        for k, v in values.items():
            setattr(self, k, v)

        self._fp16_param_init = self.fp16 or self.fp16_params

        if self.active_microbatches != self.microbatches and self.pipeline != "interleaved":
            self.pipeline = "interleaved"
            values["pipeline"] = "interleaved"
            logger.info(
                "Simple pipeline requires active_microbatches == microbatches; using interleaved pipeline."
            )
        if self.herring:
            # reference: the herring reducer raises SMPUnsupportedError (`torch/allreduce/herring.py:35-39`)
            raise SMPUnsupportedError("herring is not supported; use ddp: True (RCCL over xGMI)")
        if self.horovod:
            # the reference's PyTorch Horovod reducer (`torch/allreduce/horovod.py`) has the same
            # gradient semantics as its DDP reducer; Horovod itself is not part of this stack
            logger.warning("horovod: True -- data parallelism runs on the native RCCL reducer (as ddp: True)")
            self.ddp = True
            values["ddp"] = True
        if self.pipeline_parallel_degree > 1 and self.checkpoint_attentions:
            logger.warning("Attention checkpointing is disabled when pipeline_parallel_degree > 1.")
            self.checkpoint_attentions = False
            values["checkpoint_attentions"] = False
        self._zero2d_config_dict = {}

    # ------------------------------------------------------------ resolution
    @staticmethod
    def _default(spec, values):
        if "default" not in spec:
            raise SMPInvalidArgumentError("missing required config parameter")
        d = _eval_formula(spec["default"], values)
        if isinstance(d, (int, float)) and not isinstance(d, bool):
            if spec.get("max") is not None:
                d = min(d, _eval_formula(spec["max"], values))
            if spec.get("min") is not None:
                d = max(d, _eval_formula(spec["min"], values))
        return d

    def _validate(self, key, spec, value, values):
        types = spec.get("type")
        if types is not None:
            allowed = [_TYPES[t] for t in (types if isinstance(types, list) else [types])]
            if type(value) not in allowed:
                raise SMPConfigTypeError(
                    f"Config parameter {key} type needs to be one of {[t.__name__ for t in allowed]}. "
                    f"Found: {type(value).__name__}."
                )
        if "choices" in spec and value not in spec["choices"]:
            raise SMPInvalidArgumentError(f"Config parameter {key} must be one of {spec['choices']}. Found: {value}.")
        if value is not None and spec.get("min") is not None:
            lo = _eval_formula(spec["min"], values)
            if value < lo:
                raise SMPInvalidArgumentError(f"Config parameter {key} ({value}) cannot be less than {lo}.")
        if value is not None and spec.get("max") is not None:
            hi = _eval_formula(spec["max"], values)
            if hi is not None and value > hi:
                raise SMPInvalidArgumentError(f"Config parameter {key} ({value}) cannot be larger than {hi}.")
        default = self._default(spec, values)
        if value != default:
            for k, v in (spec.get("needs") or {}).items():
                if values[k] != v:
                    raise SMPInvalidArgumentError(
                        f"Setting config parameter {key} to non-default value {value} requires {k} to be set to {v}. "
                        f"Found: {values[k]}"
                    )
            for k, v in (spec.get("needs_not") or {}).items():
                if values[k] == v:
                    raise SMPInvalidArgumentError(
                        f"Setting config parameter {key} to non-default value {value} requires {k} to not be {v}."
                    )
            any_of = spec.get("needs_any") or {}
            if any_of and not any(values[k] == v for k, v in any_of.items()):
                raise SMPInvalidArgumentError(
                    f"Setting config parameter {key} to non-default value {value} requires either of {any_of}."
                )
        return value

    # ---------------------------------------------------------------- public
    def zero2d_enabled(self):
        return self.sharded_data_parallel_degree > 1

    def zero2d_config_dict(self):
        return self._zero2d_config_dict

    def construct_zero2d_config_dict(self, core):
        from .zero_config import construct_zero2d_config_dict

        self._zero2d_config_dict = construct_zero2d_config_dict(self, core)

    def get_config_dict(self):
        return {k: getattr(self, k) for k in self._values}

    def display_config(self):
        logger.info("Configuration parameters:")
        for k, spec in self._schema.items():
            if not spec.get("internal", False):
                logger.info(f"  {k}: {getattr(self, k)}")
        for k, spec in self._schema.items():
            if spec.get("deprecated") and k in self._input_config:
                repl = spec.get("replaced_by")
                if repl:
                    logger.warning(f'WARNING: "{k}" is a deprecated config key, please use "{repl}" instead')
                else:
                    logger.warning(f'WARNING: "{k}" is a deprecated config key')
