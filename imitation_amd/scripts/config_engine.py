"""A small, Sacred-compatible experiment/config engine.

The reference's scripts are Sacred experiments (``sacred`` is not available on the
MI355X image). This module implements the subset they rely on, with the same
user-facing behaviour:

* ``Ingredient`` / ``Experiment`` with ``@config`` scopes (plain functions whose
  local variables become config entries; scopes with parameters receive the
  current config values and may mutate them), ``@named_config`` scopes,
  ``add_named_config(name, json_path)``, ``@config_hook``, ``@capture``
  (missing arguments are filled from the ingredient's config; ``_run``, ``_rnd``,
  ``_seed``, ``_config``, ``_log`` are injected), ``@command`` / ``@main``.
* Command line: ``prog <command> [with] [named_config ...] [key.path=value ...]``,
  ``print_config``, ``-F/--file_storage DIR``, ``-n/--name``.
* Precedence exactly as in Sacred: command-line updates > named configs > config
  scopes. Values set on the command line are *fixed*: a config scope that assigns
  them keeps the fixed value, and later expressions in the scope see it.
* ``FileStorageObserver`` writing ``<dir>/<run_id>/{config.json,run.json,cout.txt}``
  plus copied artifacts -- the layout the reference's analysis tooling reads.
"""

from __future__ import annotations

import ast
import contextlib
import copy
import datetime
import functools
import hashlib
import inspect
import io
import json
import logging
import os
import pathlib
import shutil
import sys
import textwrap
import traceback
from typing import Any, Callable, Dict, Iterable, List, Mapping, Optional, Sequence, Tuple

import numpy as np

_CURRENT_RUN: Optional["Run"] = None


# --------------------------------------------------------------------------- dict helpers
def get_by_dotted_path(d: Mapping, path: str, default=None):
    if not path:
        return d
    cur: Any = d
    for part in path.split("."):
        if not isinstance(cur, Mapping) or part not in cur:
            return default
        cur = cur[part]
    return cur


def set_by_dotted_path(d: Dict, path: str, value) -> None:
    parts = path.split(".")
    cur = d
    for part in parts[:-1]:
        if not isinstance(cur.get(part), dict):
            cur[part] = {}
        cur = cur[part]
    cur[parts[-1]] = value


def recursive_update(base: Dict, upd: Mapping) -> Dict:
    """Merge ``upd`` into ``base`` in place (dicts merged recursively, others replaced)."""
    for k, v in upd.items():
        if isinstance(v, Mapping) and isinstance(base.get(k), dict):
            recursive_update(base[k], v)
        else:
            base[k] = copy.deepcopy(v)
    return base


def _jsonable(v):
    if isinstance(v, Mapping):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if isinstance(v, type) or callable(v):
        return {"py/object": f"{getattr(v, '__module__', '?')}.{getattr(v, '__qualname__', repr(v))}"}
    return repr(v)


# --------------------------------------------------------------------------- config scopes
class _FixedNamespace(dict):
    """Exec namespace: assignments to fixed keys keep the fixed value (dicts are merged
    with the fixed entries taking precedence)."""

    def __init__(self, fixed: Mapping, preset: Mapping):
        super().__init__()
        self.fixed = fixed
        for k, v in preset.items():
            dict.__setitem__(self, k, copy.deepcopy(v))
        for k, v in fixed.items():
            self.__setitem__(k, v) if k not in self else self.__setitem__(k, self[k])

    def __setitem__(self, key, value):
        if key in self.fixed:
            fv = self.fixed[key]
            if isinstance(fv, Mapping) and isinstance(value, Mapping):
                value = recursive_update(copy.deepcopy(dict(value)), fv)
            else:
                value = copy.deepcopy(fv)
        dict.__setitem__(self, key, value)

    def update(self, *args, **kwargs):  # locals().update(**SHARED) in named configs
        for k, v in dict(*args, **kwargs).items():
            self[k] = v


class ConfigScope:
    """A config function (see module docstring). Its body is executed with its parameters
    bound to the current config values; every local it ends up with becomes a config entry
    (so parameters may be mutated or re-assigned, as in Sacred)."""

    def __init__(self, func: Callable):
        self.func = func
        self.params = [p for p in inspect.signature(func).parameters]
        src = textwrap.dedent(inspect.getsource(func))
        tree = ast.parse(src)
        fdef = tree.body[0]
        assert isinstance(fdef, ast.FunctionDef)
        body = ast.Module(body=fdef.body, type_ignores=[])
        self._code = compile(body, filename=inspect.getsourcefile(func) or "<config>", mode="exec")

    def __call__(self, fixed: Mapping, preset: Mapping, current: Mapping) -> Dict:
        bound = {p: current[p] for p in self.params if p in current}
        missing = [p for p in self.params if p not in current and p not in fixed]
        if missing:
            raise KeyError(f"config scope {self.func.__name__} needs {missing}, which are not defined yet")
        ns = _FixedNamespace(fixed, {**bound, **preset})
        g = dict(self.func.__globals__)
        exec(self._code, g, ns)
        return {k: v for k, v in ns.items() if not k.startswith("_") and not inspect.ismodule(v)}


def decode_py_types(v: Any) -> Any:
    """Resolve ``{"py/type": "module:attr"}`` class references in JSON configs (allow-listed
    to this package and torch; nothing is unpickled)."""
    if isinstance(v, Mapping):
        if set(v) == {"py/type"}:
            path = v["py/type"]
            if ":" not in path:
                mod, _, name = path.rpartition(".")
                path = f"{mod}:{name}"
            if not path.startswith(("imitation_amd.", "torch.")):
                raise ValueError(f"refusing to resolve class {path!r} from a JSON config")
            mod, _, qual = path.partition(":")
            obj = __import__(mod, fromlist=["_"])
            for part in qual.split("."):
                obj = getattr(obj, part)
            return obj
        return {k: decode_py_types(x) for k, x in v.items()}
    if isinstance(v, list):
        return [decode_py_types(x) for x in v]
    return v


class _JsonNamedConfig:
    def __init__(self, path: str):
        self.path = path

    def __call__(self, fixed, preset, current):
        with open(self.path) as f:
            data = decode_py_types(json.load(f))
        return recursive_update(data, fixed)


# --------------------------------------------------------------------------- ingredients
class Ingredient:
    def __init__(self, path: str, ingredients: Sequence["Ingredient"] = ()):
        self.path = path
        self.ingredients = list(ingredients)
        self.configs: List[ConfigScope] = []
        self.named_configs: Dict[str, Any] = {}
        self.config_hooks: List[Callable] = []
        self.commands: Dict[str, Callable] = {}
        self.captured: List[Callable] = []

    # decorators ------------------------------------------------------------
    def config(self, func: Callable) -> ConfigScope:
        scope = ConfigScope(func)
        self.configs.append(scope)
        return scope

    def named_config(self, func: Callable) -> ConfigScope:
        scope = ConfigScope(func)
        self.named_configs[func.__name__] = scope
        return scope

    def add_named_config(self, name: str, conf: Any) -> None:
        if isinstance(conf, (str, os.PathLike)):
            self.named_configs[name] = _JsonNamedConfig(str(conf))
        elif isinstance(conf, Mapping):
            data = decode_py_types(dict(conf))
            self.named_configs[name] = lambda fixed, preset, current, data=data: recursive_update(copy.deepcopy(data), fixed)
        else:
            self.named_configs[name] = ConfigScope(conf)

    def add_config(self, cfg: Mapping) -> None:
        data = dict(cfg)
        self.configs.append(lambda fixed, preset, current, data=data: recursive_update(copy.deepcopy(data), fixed))  # type: ignore

    def config_hook(self, func: Callable) -> Callable:
        self.config_hooks.append(func)
        return func

    def capture(self, func: Callable = None, prefix: Optional[str] = None):
        if func is None:
            return functools.partial(self.capture, prefix=prefix)
        ingredient = self
        sig = inspect.signature(func)

        @functools.wraps(func)
        def wrapped(*args, **kwargs):
            run = _CURRENT_RUN
            if run is None:
                return func(*args, **kwargs)
            cfg = get_by_dotted_path(run.config, ingredient.config_path, {}) or {}
            if prefix:
                cfg = get_by_dotted_path(cfg, prefix, {}) or {}
            bound = sig.bind_partial(*args, **kwargs)
            for name, p in sig.parameters.items():
                if name in bound.arguments or p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD):
                    continue
                if name == "_run":
                    kwargs[name] = run
                elif name == "_config":
                    kwargs[name] = cfg
                elif name == "_seed":
                    kwargs[name] = run.derive_seed(f"{ingredient.config_path}.{func.__name__}")
                elif name == "_rnd":
                    kwargs[name] = np.random.default_rng(run.derive_seed(f"{ingredient.config_path}.{func.__name__}"))
                elif name == "_log":
                    kwargs[name] = logging.getLogger(f"{ingredient.path}.{func.__name__}")
                elif name in cfg:
                    kwargs[name] = copy.deepcopy(cfg[name])
                elif name in run.config and p.default is inspect.Parameter.empty:
                    # another ingredient's config (Sacred exposes sub-ingredient configs by path)
                    kwargs[name] = copy.deepcopy(run.config[name])
            return func(*args, **kwargs)

        self.captured.append(wrapped)
        return wrapped

    def command(self, func: Callable = None, *, unobserved: bool = False):
        if func is None:
            return functools.partial(self.command, unobserved=unobserved)
        captured = self.capture(func)
        self.commands[func.__name__] = captured
        return captured

    # config resolution ----------------------------------------------------
    @property
    def config_path(self) -> str:
        return getattr(self, "_config_path", self.path)

    def _all_ingredients(self) -> List["Ingredient"]:
        out: List[Ingredient] = []
        for ing in self.ingredients:
            for sub in ing._all_ingredients():
                if sub not in out:
                    out.append(sub)
            if ing not in out:
                out.append(ing)
        return out

    def _gather_named(self) -> Dict[str, Tuple["Ingredient", Any]]:
        named: Dict[str, Tuple[Ingredient, Any]] = {}
        for ing in self._all_ingredients():
            for k, v in ing.named_configs.items():
                named[f"{ing.path}.{k}"] = (ing, v)
        for k, v in self.named_configs.items():
            named[k] = (self, v)
        return named


class Experiment(Ingredient):
    def __init__(self, name: str, ingredients: Sequence[Ingredient] = ()):
        super().__init__(name, ingredients)
        self._config_path = ""
        self.observers: List[Any] = []
        self.default_command: Optional[str] = None
        for ing in self._all_ingredients():
            ing._config_path = ing.path

    def main(self, func: Callable) -> Callable:
        captured = self.command(func)
        self.default_command = func.__name__
        return captured

    automain = main

    # ---------------------------------------------------------------------
    def resolve_config(self, named_configs: Sequence[str] = (), config_updates: Optional[Mapping] = None,
                       command_name: Optional[str] = None) -> Dict[str, Any]:
        fixed: Dict[str, Any] = copy.deepcopy(dict(config_updates or {}))
        named = self._gather_named()
        # 1. named configs (in order), each evaluated with the CLI updates fixed
        named_updates: Dict[str, Any] = {}
        for nc in named_configs:
            if nc in named:
                ing, scope = named[nc]
            elif os.path.isfile(nc) and nc.endswith(".json"):
                ing, scope = self, _JsonNamedConfig(nc)
            else:
                raise KeyError(f"Named config not found: {nc!r}. Available: {sorted(named)}")
            path = ing.config_path
            fixed_here = get_by_dotted_path(fixed, path, {}) if path else fixed
            current = get_by_dotted_path(named_updates, path, {}) if path else named_updates
            res = scope(fixed_here or {}, {}, copy.deepcopy(current or {}))
            target = named_updates if not path else _ensure(named_updates, path)
            recursive_update(target, res)
        # CLI updates take precedence over named configs
        fixed_all = recursive_update(named_updates, fixed)
        # 2. config scopes: ingredients (depth-first), then the experiment
        config: Dict[str, Any] = {}
        for ing in self._all_ingredients() + [self]:
            path = ing.config_path
            fixed_here = (get_by_dotted_path(fixed_all, path, {}) if path else fixed_all) or {}
            cur = _ensure(config, path) if path else config
            for scope in ing.configs:
                # parameters may name entries of this ingredient or (for the experiment)
                # whole ingredient configs; they are passed by reference so that in-place
                # mutation works like in Sacred
                view = dict(config) if not path else dict(cur)
                res = scope(fixed_here, {}, view)
                recursive_update(cur, res)
            recursive_update(cur, fixed_here)
        recursive_update(config, fixed_all)
        # 3. config hooks; their updates rank below the command-line / named-config updates
        #    (Sacred: ``recursive_update(hook_updates, config_updates)``)
        for ing in self._all_ingredients() + [self]:
            path = ing.config_path
            hook_updates: Dict[str, Any] = {}
            for hook in ing.config_hooks:
                upd = hook(copy.deepcopy(config), command_name, logging.getLogger(ing.path))
                if upd:
                    recursive_update(hook_updates, upd)
            if hook_updates:
                fixed_here = (get_by_dotted_path(fixed_all, path, {}) if path else fixed_all) or {}
                recursive_update(hook_updates, fixed_here)
                recursive_update(_ensure(config, path) if path else config, hook_updates)
        if "seed" not in config:
            config["seed"] = int(np.random.SeedSequence().generate_state(1)[0] % (2**31 - 1))
        return config

    def run(self, command_name: Optional[str] = None, config_updates: Optional[Mapping] = None,
            named_configs: Sequence[str] = (), options: Optional[Mapping] = None) -> "Run":
        options = dict(options or {})
        command_name = command_name or self.default_command
        if command_name is None:
            raise ValueError("No command given and no default (@main) command defined.")
        config = self.resolve_config(named_configs, config_updates, command_name)
        if command_name == "print_config":
            run = Run(self, "print_config", config, named_configs, config_updates or {}, [])
            run.result = print_config(run)
            return run
        if command_name not in self._all_commands():
            raise KeyError(f"Unknown command {command_name!r}; available: {sorted(self._all_commands())}")
        observers = list(self.observers)
        run = Run(self, command_name, config, named_configs, config_updates or {}, observers)
        if options.get("name"):
            run.experiment_info["name"] = options["name"]
        run(self._all_commands()[command_name])
        return run

    def _all_commands(self) -> Dict[str, Callable]:
        cmds: Dict[str, Callable] = {}
        for ing in self._all_ingredients():
            cmds.update({f"{ing.path}.{k}": v for k, v in ing.commands.items()})
        cmds.update(self.commands)
        return cmds

    def run_commandline(self, argv: Optional[Sequence[str]] = None) -> Optional["Run"]:
        argv = list(sys.argv[1:] if argv is None else argv)
        command, named, updates, opts = parse_command_line(argv, set(self._all_commands()) | {"print_config"})
        if opts.get("file_storage"):
            self.observers.append(FileStorageObserver(opts["file_storage"]))
        if opts.get("help"):
            print(self.help_text())
            return None
        if opts.get("print_config") and command != "print_config":
            print_config_dict(self.resolve_config(named, updates, command))
        return self.run(command, updates, named, options=opts)

    def help_text(self) -> str:
        lines = [f"{self.path} commands:"]
        for name, fn in sorted(self._all_commands().items()):
            doc = (inspect.getdoc(fn) or "").split("\n")[0]
            lines.append(f"  {name:30s} {doc}")
        lines.append("named configs:")
        for name in sorted(self._gather_named()):
            lines.append(f"  {name}")
        return "\n".join(lines)


def _ensure(d: Dict, path: str) -> Dict:
    cur = d
    for part in path.split("."):
        if not isinstance(cur.get(part), dict):
            cur[part] = {}
        cur = cur[part]
    return cur


# --------------------------------------------------------------------------- runs & observers
class Run:
    _next_id = 1

    def __init__(self, experiment: Experiment, command: str, config: Dict, named_configs, config_updates, observers):
        self.experiment = experiment
        self.experiment_info = {"name": experiment.path}
        self.command = command
        self.config = config
        self.named_configs = list(named_configs)
        self.config_updates = dict(config_updates)
        self.observers = observers
        self.info: Dict[str, Any] = {}
        self.result: Any = None
        self.status = "INITIALIZED"
        self._id: Any = None
        self.start_time = None
        self.stop_time = None
        self.artifacts: List[str] = []
        self.metrics: Dict[str, List[Tuple[int, float]]] = {}
        self.main_function = None

    def derive_seed(self, name: str) -> int:
        h = hashlib.sha256(f"{self.config.get('seed', 0)}:{name}".encode()).digest()
        return int.from_bytes(h[:4], "little") % (2**31 - 1)

    def __call__(self, fn: Callable):
        global _CURRENT_RUN
        self.start_time = datetime.datetime.utcnow()
        self.status = "RUNNING"
        for obs in self.observers:
            self._id = obs.started_event(self)
        prev = _CURRENT_RUN
        _CURRENT_RUN = self
        capture = _Tee() if self.observers else contextlib.nullcontext()
        try:
            np.random.seed(self.config["seed"] % (2**32 - 1))
            import torch

            torch.manual_seed(self.config["seed"])
            with capture:
                self.result = fn()
            self.status = "COMPLETED"
        except BaseException as e:
            self.status = "INTERRUPTED" if isinstance(e, KeyboardInterrupt) else "FAILED"
            self.fail_trace = traceback.format_exc()
            raise
        finally:
            _CURRENT_RUN = prev
            self.stop_time = datetime.datetime.utcnow()
            for obs in self.observers:
                obs.finished_event(self, getattr(capture, "text", ""))
        return self.result

    def add_artifact(self, filename, name: Optional[str] = None) -> None:
        self.artifacts.append(str(filename))
        for obs in self.observers:
            obs.artifact_event(self, str(filename), name)

    def log_scalar(self, metric_name: str, value: float, step: Optional[int] = None) -> None:
        series = self.metrics.setdefault(metric_name, [])
        series.append((len(series) if step is None else step, float(value)))


class _Tee:
    def __init__(self):
        self.buf = io.StringIO()
        self.text = ""

    def __enter__(self):
        self._stdout = sys.stdout

        class _W:
            def __init__(s, a, b):
                s.a, s.b = a, b

            def write(s, x):
                s.a.write(x)
                s.b.write(x)
                return len(x)

            def flush(s):
                s.a.flush()

            def __getattr__(s, k):
                return getattr(s.a, k)

        sys.stdout = _W(self._stdout, self.buf)
        return self

    def __exit__(self, *exc):
        sys.stdout = self._stdout
        self.text = self.buf.getvalue()


class FileStorageObserver:
    """``<basedir>/<id>/config.json|run.json|cout.txt|metrics.json`` + artifacts (Sacred layout)."""

    def __init__(self, basedir):
        self.basedir = pathlib.Path(basedir)

    def started_event(self, run: Run):
        self.basedir.mkdir(parents=True, exist_ok=True)
        existing = [int(p.name) for p in self.basedir.iterdir() if p.is_dir() and p.name.isdigit()]
        run_id = max(existing, default=0) + 1
        d = self.basedir / str(run_id)
        d.mkdir()
        self.dir = d
        with open(d / "config.json", "w") as f:
            json.dump(_jsonable(run.config), f, indent=2, sort_keys=True)
        self._write_run(run)
        return run_id

    def _write_run(self, run: Run) -> None:
        info = {
            "experiment": run.experiment_info,
            "command": run.command,
            "status": run.status,
            "start_time": run.start_time.isoformat() if run.start_time else None,
            "stop_time": run.stop_time.isoformat() if run.stop_time else None,
            "meta": {"command": run.command, "named_configs": run.named_configs,
                     "config_updates": _jsonable(run.config_updates)},
            "result": _jsonable(run.result),
            "artifacts": [os.path.basename(a) for a in run.artifacts],
            "info": _jsonable(run.info),
        }
        if getattr(run, "fail_trace", None):
            info["fail_trace"] = run.fail_trace
        with open(self.dir / "run.json", "w") as f:
            json.dump(info, f, indent=2)

    def finished_event(self, run: Run, captured_out: str) -> None:
        with open(self.dir / "cout.txt", "w") as f:
            f.write(captured_out)
        with open(self.dir / "metrics.json", "w") as f:
            json.dump({k: {"steps": [s for s, _ in v], "values": [x for _, x in v]} for k, v in run.metrics.items()}, f)
        self._write_run(run)

    def artifact_event(self, run: Run, filename: str, name: Optional[str]) -> None:
        shutil.copy(filename, self.dir / (name or os.path.basename(filename)))


# --------------------------------------------------------------------------- command line
def _parse_value(text: str):
    try:
        return ast.literal_eval(text)
    except (ValueError, SyntaxError):
        low = text.lower()
        if low in ("true", "false"):
            return low == "true"
        if low in ("none", "null"):
            return None
        return text


#: Sacred's run options (``sacred/commandline_options.py``) accepted before ``with``.
SACRED_RUN_OPTIONS = frozenset({
    "name", "capture", "unobserved", "force", "comment", "loglevel", "id", "debug", "pdb", "beat_interval",
    "queue", "priority", "enforce_clean", "print_config", "help", "file_storage", "mongo_db", "sql", "s3",
    "tiny_db", "sacred_only", "config", "option",
})


def parse_command_line(argv: Sequence[str], commands: Iterable[str]) -> Tuple[Optional[str], List[str], Dict, Dict]:
    commands = set(commands)
    command = None
    named: List[str] = []
    updates: Dict[str, Any] = {}
    opts: Dict[str, Any] = {}
    args = list(argv)
    i = 0
    seen_with = False
    while i < len(args):
        a = args[i]
        if a in ("-F", "--file_storage"):
            opts["file_storage"] = args[i + 1]
            i += 2
            continue
        if a.startswith("--file_storage="):
            opts["file_storage"] = a.split("=", 1)[1]
        elif a in ("-p", "--print_config"):
            opts["print_config"] = True
        elif a in ("-h", "--help", "help"):
            opts["help"] = True
        elif a in ("-n", "--name"):
            opts["name"] = args[i + 1]
            i += 1
        elif a in ("-C", "--capture"):  # Sacred's output-capture mode (accepted; stdout is tee'd anyway)
            opts["capture"] = args[i + 1]
            i += 1
        elif a.startswith("--") and not seen_with:
            # another Sacred run option (--name=run0, --capture=sys, --unobserved, ...): an option,
            # never a config update; anything else is an error, as Sacred rejects unknown flags
            # (a typo such as --print-config must not be ignored silently)
            key, _, val = a[2:].partition("=")
            if key not in SACRED_RUN_OPTIONS:
                raise ValueError(f"unknown command-line option {a!r} (known: "
                                 f"{', '.join('--' + o for o in sorted(SACRED_RUN_OPTIONS))})")
            opts[key] = val if _ else True
        elif a == "with":
            seen_with = True
        elif command is None and not seen_with and a in commands:
            command = a
        elif "=" in a:
            k, v = a.split("=", 1)
            set_by_dotted_path(updates, k.strip(), _parse_value(v))
        else:
            named.append(a)
        i += 1
    return command, named, updates, opts


def print_config_dict(config: Mapping, indent: int = 0) -> str:
    lines: List[str] = []

    def rec(d: Mapping, ind: int):
        for k in sorted(d):
            v = d[k]
            if isinstance(v, Mapping) and v:
                lines.append(" " * ind + f"{k}:")
                rec(v, ind + 2)
            else:
                lines.append(" " * ind + f"{k} = {v!r}")

    rec(config, indent)
    text = "Configuration:\n" + "\n".join(lines)
    print(text)
    return text


def print_config(run: Run) -> str:
    return print_config_dict(run.config)


def current_run() -> Optional[Run]:
    return _CURRENT_RUN
