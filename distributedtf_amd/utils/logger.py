"""Benchmark / metric logger (reference ``official/utils/logs/logger.py``).

* ``BaseBenchmarkLogger``  -- metrics as JSON on stdout (python ``logging``);
* ``BenchmarkFileLogger``  -- JSON lines in ``<dir>/metric.log`` + ``benchmark_run.log``;
* ``config_benchmark_logger`` / ``get_benchmark_logger`` -- process-wide logger behind a lock;
* ``benchmark_context``    -- records success / failure of a run.
Run info collects ROCm / HIP / torch versions, the GPU (name, count, HBM size)
and host CPU / memory instead of TF / GCP fields (BigQuery upload is not part of
this build: no network).
"""

from __future__ import annotations

import contextlib
import datetime
import json
import logging
import numbers
import os
import platform
import threading
from typing import Any, Dict, Optional

METRIC_LOG_FILE_NAME = "metric.log"
BENCHMARK_RUN_LOG_FILE_NAME = "benchmark_run.log"
_DATE_TIME_FORMAT_PATTERN = "%Y-%m-%dT%H:%M:%S.%fZ"
RUN_STATUS_SUCCESS = "success"
RUN_STATUS_FAILURE = "failure"
RUN_STATUS_RUNNING = "running"

log = logging.getLogger("distributedtf_amd")
_logger_lock = threading.Lock()
_benchmark_logger = None


def _process_metric_to_json(name, value, unit=None, global_step=None, extras=None) -> Optional[Dict[str, Any]]:
    if not isinstance(value, numbers.Number) or isinstance(value, bool):
        log.warning("Metric value to log should be a number. Got %s", type(value))
        return None
    extras = [{"name": k, "value": v} for k, v in sorted((extras or {}).items())]
    return {"name": name, "value": float(value), "unit": unit, "global_step": global_step,
            "timestamp": datetime.datetime.utcnow().strftime(_DATE_TIME_FORMAT_PATTERN), "extras": extras}


def _rocm_version() -> Optional[str]:
    for p in ("/opt/rocm/.info/version", "/opt/rocm/.info/version-dev"):
        try:
            with open(p) as f:
                return f.read().strip()
        except OSError:
            continue
    return None


def gather_run_info(model_name, dataset_name, run_params, test_id=None) -> Dict[str, Any]:
    info: Dict[str, Any] = {"model_name": model_name, "dataset": {"name": dataset_name},
                            "machine_config": {}, "test_id": test_id,
                            "run_date": datetime.datetime.utcnow().strftime(_DATE_TIME_FORMAT_PATTERN)}
    try:
        import torch
        info["framework_version"] = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
                                     "rocm": _rocm_version()}
        if torch.cuda.is_available():
            props = torch.cuda.get_device_properties(0)
            info["machine_config"]["gpu_info"] = {"count": torch.cuda.device_count(), "model": props.name,
                                                  "hbm_bytes": int(props.total_memory),
                                                  "arch": getattr(props, "gcnArchName", None)}
    except Exception:  # pragma: no cover
        pass
    info["machine_config"]["cpu_info"] = {"num_cores": os.cpu_count(), "cpu_info": platform.processor()}
    try:
        import psutil
        vm = psutil.virtual_memory()
        info["machine_config"]["memory_total"] = vm.total
        info["machine_config"]["memory_available"] = vm.available
    except Exception:  # pragma: no cover
        pass
    info["run_parameters"] = [{"name": k, "value": v if isinstance(v, (int, float, str, bool)) or v is None else str(v)}
                              for k, v in sorted((run_params or {}).items())]
    info["tensorflow_environment_variables"] = [{"name": k, "value": v} for k, v in sorted(os.environ.items())
                                                if k.startswith(("HIP_", "HSA_", "ROCR_", "DTF_", "NCCL_", "RCCL_"))]
    return info


class BaseBenchmarkLogger:
    def log_evaluation_result(self, eval_results: Dict[str, Any]):
        if not isinstance(eval_results, dict):
            log.warning("eval_results should be dictionary for logging. Got %s", type(eval_results))
            return
        step = eval_results.get("global_step")
        for k in sorted(eval_results):
            if k != "global_step":
                self.log_metric(k, eval_results[k], global_step=step)

    def log_metric(self, name, value, unit=None, global_step=None, extras=None):
        m = _process_metric_to_json(name, value, unit, global_step, extras)
        if m:
            log.info("Benchmark metric: %s", m)
        return m

    def log_run_info(self, model_name, dataset_name, run_params, test_id=None):
        info = gather_run_info(model_name, dataset_name, run_params, test_id)
        log.info("Benchmark run: %s", info)
        return info

    def on_finish(self, status):
        pass


class BenchmarkFileLogger(BaseBenchmarkLogger):
    def __init__(self, logging_dir: str):
        logging_dir = os.path.abspath(logging_dir)  # the cwd may change during a run
        self._logging_dir = logging_dir
        os.makedirs(logging_dir, exist_ok=True)
        self._metric_path = os.path.join(logging_dir, METRIC_LOG_FILE_NAME)
        self._lock = threading.Lock()

    def log_metric(self, name, value, unit=None, global_step=None, extras=None):
        m = _process_metric_to_json(name, value, unit, global_step, extras)
        if m:
            with self._lock, open(self._metric_path, "a") as f:
                f.write(json.dumps(m) + "\n")
        return m

    def log_run_info(self, model_name, dataset_name, run_params, test_id=None):
        info = gather_run_info(model_name, dataset_name, run_params, test_id)
        with open(os.path.join(self._logging_dir, BENCHMARK_RUN_LOG_FILE_NAME), "w") as f:
            json.dump(info, f)
            f.write("\n")
        return info

    def on_finish(self, status):
        path = os.path.join(self._logging_dir, BENCHMARK_RUN_LOG_FILE_NAME)
        info = {}
        if os.path.isfile(path):
            with open(path) as f:
                try:
                    info = json.load(f)
                except ValueError:
                    info = {}
        info["status"] = status
        with open(path, "w") as f:
            json.dump(info, f)
            f.write("\n")


def rank_log_dir(log_dir: str, rank: int = 0) -> str:
    """Where process ``rank`` of a multi-process run writes its benchmark files: rank 0 (and a single-process run)
    the directory itself, rank k > 0 ``<dir>/rank_<k>`` -- every training process logs its own members' eval
    results, as each reference worker process does (resnet_run_loop.py:466)."""
    return log_dir if not rank else os.path.join(log_dir, "rank_%d" % int(rank))


def config_benchmark_logger(flag_obj=None, rank: int = 0):
    """``benchmark_logger_type`` in {BaseBenchmarkLogger, BenchmarkFileLogger} (+ ``benchmark_log_dir``);
    ``rank`` picks the per-process directory (``rank_log_dir``)."""
    global _benchmark_logger
    with _logger_lock:
        kind = getattr(flag_obj, "benchmark_logger_type", "BaseBenchmarkLogger") if flag_obj else "BaseBenchmarkLogger"
        if kind == "BaseBenchmarkLogger":
            _benchmark_logger = BaseBenchmarkLogger()
        elif kind == "BenchmarkFileLogger":
            d = getattr(flag_obj, "benchmark_log_dir", None)
            if not d:
                raise ValueError("BenchmarkFileLogger needs benchmark_log_dir")
            _benchmark_logger = BenchmarkFileLogger(rank_log_dir(d, rank))
        else:
            raise ValueError("Unrecognized benchmark_logger_type: %s" % kind)
    return _benchmark_logger


def get_benchmark_logger():
    if _benchmark_logger is None:
        config_benchmark_logger(None)
    return _benchmark_logger


@contextlib.contextmanager
def benchmark_context(flag_obj=None, rank: int = 0):
    """Configure the process-wide logger for one run; the previous logger is restored afterwards."""
    global _benchmark_logger
    prev = _benchmark_logger
    bl = config_benchmark_logger(flag_obj, rank=rank)
    try:
        yield bl
        bl.on_finish(RUN_STATUS_SUCCESS)
    except Exception:
        bl.on_finish(RUN_STATUS_FAILURE)
        raise
    finally:
        with _logger_lock:
            _benchmark_logger = prev
