"""Small helpers: timing, formatting, environment probes."""
from __future__ import annotations

import json
import os
import time
from contextlib import contextmanager
from typing import Iterator


@contextmanager
def wall_timer() -> Iterator[dict]:
    """``with wall_timer() as t: ...`` then ``t["seconds"]`` (host steady clock).

    Replaces the reference's dead ``cpuSecond()`` helper (CUDACG.cu:35-39), which
    was defined but never called."""
    box = {"seconds": 0.0}
    t0 = time.perf_counter()
    try:
        yield box
    finally:
        box["seconds"] = time.perf_counter() - t0


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def json_line(obj: dict) -> str:
    return json.dumps(obj, separators=(", ", ": "))


def env_flag(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


def format_x(x) -> str:
    """The reference's output format: one ``%f`` per line (CUDACG.cu:361-364)."""
    return "".join("%f\n" % float(v) for v in x)
