"""Pass-through command-line options for lab processors.

The reference forwards every unknown ``--key value`` pair to the lab processor
constructor, coercing bool -> int -> float -> str (reference
arg_parsing.py:1-31). That coercion cannot express lists, so e.g.
``--extra_links_to_png URL`` was iterated character by character (SURVEY
Appendix B #5). Here a value that parses as JSON list/object is decoded as
JSON; everything else keeps the reference's coercion order. A bare flag is
``True``; ``--key=value`` is accepted too.
"""

from __future__ import annotations

import json
from typing import Any, Dict, List


def coerce(value: str) -> Any:
    low = value.lower()
    if low in ("true", "false"):
        return low == "true"
    s = value.strip()
    if s[:1] in "[{":
        try:
            return json.loads(s)
        except json.JSONDecodeError:
            pass
    for cast in (int, float):
        try:
            return cast(value)
        except ValueError:
            continue
    return value


def passthrough_kwargs(argv: List[str]) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    i = 0
    while i < len(argv):
        tok = argv[i]
        if tok.startswith("--") and len(tok) > 2:
            key = tok[2:]
            if "=" in key:
                key, val = key.split("=", 1)
                out[key] = coerce(val)
            elif i + 1 < len(argv) and not argv[i + 1].startswith("--"):
                out[key] = coerce(argv[i + 1])
                i += 1
            else:
                out[key] = True
        i += 1
    return out
