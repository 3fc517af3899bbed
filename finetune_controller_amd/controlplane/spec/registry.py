"""Model registry (C8): built-in specs + dynamically loaded custom model files.

``JOB_MANIFESTS`` maps a spec's ``name`` default to its class
(``/root/reference/app/jobs/registered_models.py:15-37``); ``load_models_from_directory`` imports every
``*.py`` in a directory and registers each ``BaseFineTuneModel`` subclass it defines
(``/root/reference/app/models/model_loader.py:14-45``).  Import is by file path with a unique module
name (no ``sys.path`` mutation), and a broken custom file is logged and skipped.
"""
from __future__ import annotations

import importlib.util
import logging
import os
from pathlib import Path

from .finetuning import BaseFineTuneModel
from .models.builtin import BUILTIN_MODELS

logger = logging.getLogger("ftc.registry")


def spec_name(cls) -> str:
    return cls.model_fields["name"].get_default()


def inference_name(cls) -> str | None:
    f = cls.model_fields.get("inference_name")
    return f.get_default() if f else None


def load_models_from_directory(directory: str) -> dict[str, type[BaseFineTuneModel]]:
    models: dict[str, type[BaseFineTuneModel]] = {}
    d = Path(directory)
    if not d.is_dir():
        return models
    for file in sorted(d.glob("*.py")):
        if file.name.startswith("__"):
            continue
        mod_name = f"ftc_custom_models.{file.stem}"
        try:
            spec = importlib.util.spec_from_file_location(mod_name, file)
            module = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(module)
        except Exception as e:
            logger.error("error loading model module %s: %s", file.name, e)
            continue
        for attr in vars(module).values():
            if isinstance(attr, type) and issubclass(attr, BaseFineTuneModel) and attr is not BaseFineTuneModel \
                    and attr.__module__ == mod_name:
                try:
                    spec_name(attr)
                except Exception:
                    continue  # abstract helper without a name default
                models[attr.__name__] = attr
    return models


class ModelRegistry:
    def __init__(self, include_builtin: bool = True):
        self.manifests: dict[str, type[BaseFineTuneModel]] = {}
        if include_builtin:
            for cls in BUILTIN_MODELS:
                self.manifests[spec_name(cls)] = cls

    def register(self, cls: type[BaseFineTuneModel]) -> bool:
        name = spec_name(cls)
        if name in self.manifests:
            logger.warning("model name %r already registered; skipping", name)
            return False
        self.manifests[name] = cls
        logger.info("registered model: %s", name)
        return True

    def load_custom(self, directory: str | None = None) -> int:
        directory = directory or os.environ.get("CUSTOM_MODELS_DIR") or str(Path(__file__).parent / "custom")
        n = 0
        for cls in load_models_from_directory(directory).values():
            n += self.register(cls)
        return n

    def get(self, name: str):
        return self.manifests.get(name)

    def instance(self, name: str):
        cls = self.manifests.get(name)
        return cls() if cls else None

    def names(self) -> list[str]:
        return list(self.manifests)

    def available_for(self, scopes: list[str] | None) -> list[str]:
        """Models visible to a token: those whose ``inference_name`` is in the token's ``scp`` claim
        (``/root/reference/app/main.py:1323-1341``).  ``None`` (no token) = all models."""
        if scopes is None:
            return self.names()
        return [n for n, c in self.manifests.items() if (inn := inference_name(c)) and inn in scopes]

    def all_inference_names(self) -> list[str]:
        out = []
        for c in self.manifests.values():
            n = inference_name(c)
            if n and n not in out:
                out.append(n)
        return out
