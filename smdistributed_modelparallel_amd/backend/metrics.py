"""Partition metrics publishing (reference `backend/utils.py:134-149` upload_metrics_to_studio,
called once per job from `torch/step.py:295-311`).

The reference pushes a handful of partition metrics (forward communication volume between
devices, hops between devices in the first microbatch, parameter count and module fraction
per pipeline device) to SageMaker Studio through ``smexperiments``' file metrics writer, and
warns when that package is missing.  Here the same metrics go to every sink that is
configured:

* ``smexperiments.metrics.SageMakerFileMetricsWriter`` when importable (reference path);
* ``SMP_METRICS_FILE``: one JSON object per publication appended to the file;
* ``SMP_METRICS_PROMETHEUS_FILE``: a Prometheus text-format file (node-exporter textfile
  collector), gauges named ``smp_<metric>``;
* always: one INFO log line.
"""
import json
import os
import re
import time

from .logger import get_logger

try:  # pragma: no cover - not installed in this image
    from smexperiments.metrics import SageMakerFileMetricsWriter
except Exception:  # noqa: BLE001
    SageMakerFileMetricsWriter = None


def _prom_name(name):
    s = re.sub(r"[^a-zA-Z0-9_]", "_", name).strip("_").lower()
    return "smp_" + re.sub(r"_+", "_", s)


def upload_metrics_to_studio(metrics):
    """Publish a flat {name: number} dict to the configured sinks; returns the sinks used."""
    used = []
    if SageMakerFileMetricsWriter is not None:  # pragma: no cover
        writer = SageMakerFileMetricsWriter()
        try:
            for name, value in metrics.items():
                writer.log_metric(metric_name=name, value=value)
        finally:
            writer.close()
        used.append("studio")
    path = os.environ.get("SMP_METRICS_FILE")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"time": time.time(), "metrics": metrics}, sort_keys=True) + "\n")
        used.append("file")
    prom = os.environ.get("SMP_METRICS_PROMETHEUS_FILE")
    if prom:
        from prometheus_client import CollectorRegistry, Gauge, write_to_textfile

        reg = CollectorRegistry()
        for name, value in metrics.items():
            Gauge(_prom_name(name), f"smdistributed partition metric {name}", registry=reg).set(float(value))
        write_to_textfile(prom, reg)
        used.append("prometheus")
    get_logger().info("partition metrics: " + ", ".join(f"{k}={v}" for k, v in metrics.items()))
    return used
