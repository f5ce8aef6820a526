"""Dotted-path plugin loader (reference: utils/class_utils.py:1-8).

Besides ``package.module.Class`` paths this loader accepts the reference's own
config paths unchanged, so a reference pipeline JSON runs on this framework
without edits: ``models.r2p1d.model.R2P1DLoader``, ``batcher.Batcher``,
``selector.RoundRobinSelector`` and ``video_path_provider.*`` are resolved to
their ``rnb_amd`` equivalents.
"""
from __future__ import annotations

import importlib

# reference module prefix -> rnb_amd module
_LEGACY_PREFIXES = (
    ("models.", "rnb_amd.models."),
    ("batcher.", "rnb_amd.batcher."),
    ("selector.", "rnb_amd.selector."),
    ("video_path_provider.", "rnb_amd.video_path_provider."),
    ("runner_model.", "rnb_amd.runner_model."),
)


def resolve_path(path: str) -> str:
    """Map a legacy reference dotted path onto the rnb_amd package."""
    for old, new in _LEGACY_PREFIXES:
        if path.startswith(old):
            return new + path[len(old):]
    return path


def load_class(path: str):
    """Import ``a.b.C`` and return ``C``."""
    if not isinstance(path, str) or "." not in path:
        raise ValueError("expected a dotted class path, got %r" % (path,))
    candidates = [path]
    resolved = resolve_path(path)
    if resolved != path:
        candidates.insert(0, resolved)
    last_err = None
    for cand in candidates:
        module_path, cls_name = cand.rsplit(".", 1)
        try:
            module = importlib.import_module(module_path)
        except ImportError as err:
            last_err = err
            continue
        if hasattr(module, cls_name):
            return getattr(module, cls_name)
        last_err = AttributeError("module %s has no attribute %s"
                                  % (module_path, cls_name))
    raise ImportError("cannot load class %r: %s" % (path, last_err))
