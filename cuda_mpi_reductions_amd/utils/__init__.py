"""Reference-compatible CLI grammar, output formats, averaging and plotting helpers."""
from . import cli, formats, getavgs  # noqa: F401
