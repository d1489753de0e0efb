"""Reference-compatible CLI grammar, output formats, averaging and timing helpers."""
