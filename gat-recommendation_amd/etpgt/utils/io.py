"""I/O helpers — API of etpgt/utils/io.py (reference): YAML config (safe loader) and
JSON load / save (parent directories created)."""

from __future__ import annotations

import json
from pathlib import Path
from typing import Any


def load_config(config_path: str) -> dict[str, Any]:
    import yaml

    with open(config_path) as f:
        return yaml.safe_load(f)


def save_json(data: dict[str, Any], output_path: str) -> None:
    Path(output_path).parent.mkdir(parents=True, exist_ok=True)
    with open(output_path, "w") as f:
        json.dump(data, f, indent=2)


def load_json(input_path: str) -> dict[str, Any]:
    with open(input_path) as f:
        return json.load(f)
