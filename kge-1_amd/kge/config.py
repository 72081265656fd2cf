"""Hierarchical YAML configuration: the subset of LibKGE's Config / Configurable
(kge/config.py:16-629) that the scoring path reads.

Semantics kept from the reference:
  * dotted keys ("train.batch_size"), nested dicts, "+++" marks a dict that accepts new
    keys (config.py:144-236);
  * ``_import(name)`` merges ``kge/model/<name>.yaml`` (and its ``import:`` list) the way
    Config._import does (config.py:238-281);
  * ``get_default(key)`` resolves a missing key through the ``type`` of its parent, so
    ``complex.entity_embedder.dim`` falls back to ``lookup_embedder.dim``
    (config.py:69-114);
  * ``Configurable.get_option`` reads ``<configuration_key>.<name>`` (config.py:570-629).
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, Optional

import yaml

_HERE = os.path.dirname(os.path.abspath(__file__))
_MODEL_DIRS = [os.path.join(_HERE, "model"), os.path.join(_HERE, "model", "embedder")]


def _number_or_str(v: str):
    for conv in (int, float):
        try:
            return conv(v)
        except ValueError:
            pass
    return v


def _strip_plus(d):
    if isinstance(d, dict):
        return {k: _strip_plus(v) for k, v in d.items() if k != "+++"}
    return d


class Config:
    def __init__(self, folder: Optional[str] = None, load_default: bool = True):
        if load_default:
            with open(os.path.join(_HERE, "config-default.yaml")) as f:
                self.options: Dict[str, Any] = yaml.load(f, Loader=yaml.SafeLoader)
        else:
            self.options = {}
        self.folder = folder
        self.log_folder: Optional[str] = None
        self.log_prefix: Optional[str] = None
        self._imported = set()

    # -------------------------------------------------------------------- access
    def get(self, key: str, remove_plusplusplus: bool = True) -> Any:
        node = self.options
        for name in key.split("."):
            if not isinstance(node, dict) or name not in node:
                raise KeyError(f"Error accessing {name} for key {key}")
            node = node[name]
        return _strip_plus(node) if remove_plusplusplus else node

    def exists(self, key: str) -> bool:
        try:
            self.get(key)
            return True
        except KeyError:
            return False

    def get_default(self, key: str) -> Any:
        """Value of key; if absent, resolve through the ``type`` of its parent."""
        try:
            return self.get(key)
        except KeyError as e:
            parts = key.split(".")
            for i in range(len(parts) - 1, 0, -1):
                parent = ".".join(parts[:i])
                try:
                    parent_type = self.get(parent + ".type")
                except KeyError:
                    continue
                rest = ".".join(parts[i:])
                return self.get_default(f"{parent_type}.{rest}")
            raise e

    def set(self, key: str, value, create: bool = False, overwrite: bool = True, log: bool = False):
        """Set a dotted key with the reference's checks (config.py:144-236): a key that does
        not exist yet may only be created with create=True or under a dict that carries
        "+++" (KeyError otherwise, so a misspelt option is not silently ignored), and a new
        value must have the type of the value it replaces (ValueError; numeric strings are
        converted, and an int is accepted where a float is stored)."""
        parts = key.split(".")
        node = self.options
        for i, name in enumerate(parts[:-1]):
            if name in node and isinstance(node[name], dict):
                create = create or "+++" in node[name]
            elif name in node and node[name] is not None:
                raise KeyError(f"Key '{key}' cannot be set because '{'.'.join(parts[:i + 1])}' is not a dictionary")
            else:
                if not create:
                    where = "at root level" if i == 0 else f"under key '{'.'.join(parts[:i])}'"
                    raise KeyError(f"Key '{key}' cannot be set because key '{'.'.join(parts[:i + 1])}' does not "
                                   f"exist and no new keys are allowed to be created {where}.")
                node[name] = {}
            node = node[name]
        last = parts[-1]
        old = node.get(last)
        if old is None:
            if not create:
                where = "at root level" if len(parts) == 1 else f"under key '{'.'.join(parts[:-1])}'"
                raise KeyError(f"Key '{key}' cannot be set because it does not exist and no new keys are "
                               f"allowed to be created {where}.")
            if isinstance(value, str):
                value = _number_or_str(value)
        else:
            if isinstance(value, str) and isinstance(old, (int, float)) and not isinstance(old, bool):
                conv = _number_or_str(value)
                if not isinstance(conv, str):
                    value = float(conv) if isinstance(old, float) else conv
            if isinstance(old, float) and isinstance(value, int) and not isinstance(value, bool):
                value = float(value)
            if type(value) != type(old):
                raise ValueError(f"key '{key}' has incorrect type (expected {type(old)}, found {type(value)})")
            if not overwrite:
                return old
        node[last] = value
        return value

    def set_all(self, new_options: Dict[str, Any], create: bool = False):
        for k, v in Config.flatten(new_options).items():
            self.set(k, v, create=True)

    # -------------------------------------------------------------------- import / load
    def _import(self, module_name: str):
        """Merge kge/model[/embedder]/<module_name>.yaml (and its imports)."""
        if module_name in self._imported:
            return
        fn = None
        for d in _MODEL_DIRS:
            cand = os.path.join(d, f"{module_name}.yaml")
            if os.path.exists(cand):
                fn = cand
                break
        if fn is None:
            raise ValueError(f"Module {module_name} not found")
        with open(fn) as f:
            opts = yaml.load(f, Loader=yaml.SafeLoader)
        self._imported.add(module_name)
        for imp in opts.pop("import", []) or []:
            self._import(imp)
        for top, val in opts.items():
            if top in self.options and isinstance(self.options[top], dict) and isinstance(val, dict):
                merged = copy.deepcopy(val)
                _deep_update(merged, self.options[top])
                self.options[top] = merged
            elif top not in self.options:
                self.options[top] = val

    def load(self, filename: str, create: bool = True):
        with open(filename) as f:
            opts = yaml.load(f, Loader=yaml.SafeLoader) or {}
        self.load_options(opts, create=create)

    def load_options(self, opts: Dict[str, Any], create: bool = True):
        if "model" in opts and opts["model"]:
            self._import(opts["model"])
        for imp in opts.pop("import", []) or []:
            self._import(imp)
        for k, v in Config.flatten(opts).items():
            self.set(k, v, create=create)

    @staticmethod
    def flatten(options: Dict[str, Any]) -> Dict[str, Any]:
        out: Dict[str, Any] = {}

        def rec(d, prefix):
            for k, v in d.items():
                if k == "+++":
                    continue
                key = f"{prefix}{k}"
                if isinstance(v, dict) and v:
                    rec(v, key + ".")
                else:
                    out[key] = v

        rec(options, "")
        return out

    def clone(self) -> "Config":
        c = Config(self.folder, load_default=False)
        c.options = copy.deepcopy(self.options)
        c._imported = set(self._imported)
        c.log_folder = self.log_folder
        return c

    def check(self, key: str, allowed_values) -> Any:
        v = self.get(key)
        if v not in allowed_values:
            raise ValueError(f"Illegal value {v} for key {key}; allowed values are {allowed_values}")
        return v

    def log(self, msg: str, echo: bool = True, prefix: str = ""):
        if echo and self.get("verbose"):
            print(prefix + msg)

    def print(self, *args, **kwargs):
        if self.get("verbose"):
            print(*args, **kwargs)


def _deep_update(target: dict, src: dict):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(target.get(k), dict):
            _deep_update(target[k], v)
        else:
            target[k] = copy.deepcopy(v)


class Configurable:
    """Mix-in for objects configured under a key (config.py:570-629)."""

    def __init__(self, config: Config, configuration_key: Optional[str] = None):
        self._init_configuration(config, configuration_key)

    def _init_configuration(self, config: Config, configuration_key: Optional[str]):
        self.config = config
        self.configuration_key = configuration_key

    def _key(self, name: str) -> str:
        return f"{self.configuration_key}.{name}" if self.configuration_key else name

    def has_option(self, name: str) -> bool:
        try:
            self.get_option(name)
            return True
        except KeyError:
            return False

    def get_option(self, name: str) -> Any:
        return self.config.get_default(self._key(name))

    def check_option(self, name: str, allowed_values) -> Any:
        v = self.get_option(name)
        if v not in allowed_values:
            raise ValueError(f"Illegal value {v} for key {self._key(name)}; allowed values are {allowed_values}")
        return v

    def set_option(self, name: str, value, create: bool = False, log: bool = False):
        return self.config.set(self._key(name), value, create=True)
