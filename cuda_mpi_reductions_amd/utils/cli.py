"""The SDK command-line grammar (CmdArgReader, cuda/C/common/src/cmd_arg_reader.cpp:119-151) in
Python, for Python front-ends that must accept the reference's flags verbatim: every token starts
with ``-``; ``-name``/``--name`` is a flag; ``-name=value``/``--name=value`` sets a value. The C++
apps use the identical csrc/runtime/cli.cpp."""
from __future__ import annotations

from typing import Dict, List, Optional

FLAG = object()


class CliError(ValueError):
    pass


def parse(argv: List[str]) -> Dict[str, object]:
    args: Dict[str, object] = {}
    for a in argv:
        if not a or a[0] != "-":
            raise CliError(f"Invalid command line argument: {a!r} (arguments must start with - or --)")
        dashes = 2 if len(a) > 1 and a[1] == "-" else 1
        if "=" in a:
            k, v = a[dashes:].split("=", 1)
            args[k] = v
        else:
            args[a[dashes:]] = FLAG
    return args


def parse_count(s: str) -> int:
    """Integers with k/M/G (2^10/2^20/2^30) suffixes or e-notation ("1e9")."""
    s = s.strip()
    mult = {"k": 1 << 10, "K": 1 << 10, "m": 1 << 20, "M": 1 << 20, "g": 1 << 30, "G": 1 << 30}
    if s and s[-1] in mult:
        return int(s[:-1]) * mult[s[-1]]
    if "e" in s or "E" in s:
        v = float(s)
        if v != int(v) or v < 0:
            raise CliError(f"not a count: {s}")
        return int(v)
    return int(s)


def get_str(args: Dict[str, object], name: str) -> Optional[str]:
    v = args.get(name)
    return None if v is None or v is FLAG else str(v)


def get_int(args: Dict[str, object], name: str, default: Optional[int] = None) -> Optional[int]:
    v = get_str(args, name)
    return default if v is None else parse_count(v)


def has(args: Dict[str, object], name: str) -> bool:
    return name in args
