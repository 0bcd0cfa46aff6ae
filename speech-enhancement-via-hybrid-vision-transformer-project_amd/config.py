"""YAML configuration loading for the enhance / train call surface
(the reference's utils/config.py, which its enhance.py imports at :20 but its
utils/__init__.py does not export -- SURVEY §3.C).

``load_all_configs(config_dir)`` merges ``data_config.yaml``,
``model_config.yaml`` and ``train_config.yaml`` in that order
(utils/config.py:77-110): a later file's keys win, nested dicts merge key by
key (merge_configs, :51-74), and a missing file is reported and skipped; a
missing directory raises FileNotFoundError.  ``yaml.safe_load`` only.
"""

from __future__ import annotations

from pathlib import Path
from typing import Any, Dict, Union

CONFIG_FILES = ("data_config.yaml", "model_config.yaml", "train_config.yaml")


def load_config(config_path: Union[str, Path]) -> Dict[str, Any]:
    """utils/config.py:16-32: one YAML file (FileNotFoundError if absent)."""
    import yaml

    p = Path(config_path)
    if not p.exists():
        raise FileNotFoundError(f"Configuration file not found: {p}")
    with open(p) as f:
        return yaml.safe_load(f)


def merge_configs(base_config: Dict, override_config: Dict) -> Dict:
    """utils/config.py:51-74: override wins; dicts present on both sides merge
    recursively; the inputs are not modified."""
    out = dict(base_config)
    for k, v in (override_config or {}).items():
        if isinstance(out.get(k), dict) and isinstance(v, dict):
            out[k] = merge_configs(out[k], v)
        else:
            out[k] = v
    return out


def load_all_configs(config_dir: Union[str, Path] = "config") -> Dict[str, Any]:
    """utils/config.py:77-110."""
    d = Path(config_dir)
    if not d.exists():
        raise FileNotFoundError(f"Configuration directory not found: {d}")
    merged: Dict[str, Any] = {}
    for name in CONFIG_FILES:
        p = d / name
        if p.exists():
            merged = merge_configs(merged, load_config(p) or {})
        else:
            print(f"Warning: Configuration file not found: {p}")
    return merged


__all__ = ["load_config", "merge_configs", "load_all_configs"]
