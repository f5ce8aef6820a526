"""Utilities: plugin loading, argparse validators, device discovery."""
from .class_utils import load_class, resolve_path  # noqa: F401
