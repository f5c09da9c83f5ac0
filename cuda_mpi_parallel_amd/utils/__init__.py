"""Output helpers shared by the entry points (CLI, bench.py, smoke test, tests)."""
from __future__ import annotations

import json
from typing import Iterable, Optional


def format_x(x: Iterable[float]) -> str:
    """The reference's solution output: one ``%f`` per line (CUDACG.cu:361-364)."""
    return "".join("%f\n" % float(v) for v in x)


def last_json_line(text: str) -> Optional[dict]:
    """The last line of ``text`` that parses as a JSON object (bench / ``--report json`` output,
    which may follow library banners on the same stream); None when there is none."""
    for line in reversed(text.strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None
