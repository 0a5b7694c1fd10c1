"""Minimal stand-in for gymnasium (not installed here) so the reference env imports.
Only used by tools/oracle fixture generation in the dev container; never shipped."""
from . import spaces  # noqa: F401
