"""Configuration: one layered key/value tree, HOCON-compatible input.

The reference takes settings from three places: positional CLI args,
constants hard-coded in `AllreduceMaster.main` (AllreduceMaster.scala:105-114) and HOCON
files (`application.conf`, test `reference.conf`). Here every setting lives under `mxar.*`
with the same defaults, layered (later wins):

    built-in defaults  <  config file(s)  <  MXAR_* environment  <  CLI --set key=value

The file parser reads the HOCON subset the reference's files use (nested `{}` blocks,
dotted keys, `=`/`:`, quoted/unquoted strings, numbers, booleans, `[...]` lists, `#`/`//`
comments, duration values like `10s`/`500ms`). The reference's own `akka.*` keys are
accepted as aliases, so its `application.conf` can be pointed at this framework as is.
"""
from __future__ import annotations

import copy
import os
import re
from typing import Any, Iterable

DEFAULTS: dict[str, Any] = {
    "mxar.system-name": "ClusterSystem",                       # AllreduceMaster.scala:120
    "mxar.remote.hostname": "127.0.0.1",                       # application.conf:8
    "mxar.remote.port": 0,
    "mxar.cluster.seed-nodes": ["mxar.tcp://ClusterSystem@127.0.0.1:2551",
                                "mxar.tcp://ClusterSystem@127.0.0.1:2552"],  # application.conf:14-16
    "mxar.cluster.roles": [],
    "mxar.cluster.auto-down-unreachable-after": 10.0,          # application.conf:20 (seconds)
    "mxar.cluster.failure-detector.heartbeat-interval": 1.0,
    "mxar.cluster.failure-detector.acceptable-heartbeat-pause": 3.0,
    "mxar.cluster.worker-path": "/user/worker",                # AllreduceMaster.scala:73
    "mxar.loglevel": "INFO",                                   # application.conf:22
    "mxar.log-dead-letters": 5,                                # application.conf:23
    "mxar.allreduce.total-workers": 2,                         # AllreduceMaster.scala:112
    "mxar.allreduce.data-size": 10,                            # totalWorkers * 5
    "mxar.allreduce.max-chunk-size": 2,                        # AllreduceMaster.scala:114
    "mxar.allreduce.th-allreduce": 1.0,                        # AllreduceMaster.scala:105
    "mxar.allreduce.th-reduce": 0.9,                           # :106
    "mxar.allreduce.th-complete": 0.8,                         # :107
    "mxar.allreduce.max-lag": 1,                               # :108
    "mxar.allreduce.max-round": 100,                           # :109
    "mxar.allreduce.live-barrier": False,
    "mxar.allreduce.reinit-on-loss": False,                    # re-init the survivors when a worker dies
    "mxar.allreduce.resume-on-join": False,                    # a mid-job join resumes everyone at the current round
    "mxar.bridge.port": -1,                                    # control bridge TCP port (-1 off, 0 any free port)
    "mxar.bridge.host": "127.0.0.1",                           # control bridge listen address
    "mxar.bridge.external-rounds": False,                      # bridge clients drive the rounds (StartAllreduce)
    "mxar.akka.port": -1,                                      # akka.tcp endpoint of the master (-1 off; docs/AKKA_WIRE.md)
    "mxar.akka.package": "sample.cluster.allreduce",           # package of the message classes (AllreduceMessage.scala:1)
    "mxar.akka.cookie": "",                                    # akka.remote.require-cookie (empty: none)
    "mxar.akka.suid.start-allreduce": 0,                       # serialVersionUID overrides (0: scalac 2.12 model)
    "mxar.akka.suid.complete-allreduce": 0,
    "mxar.allreduce.round-timeout": 0.0,                       # seconds; 0 = off
    "mxar.engine.device": "cpu",                               # cpu | cuda[:i]
    "mxar.engine.algo": "auto",                                # auto | twoshot | oneshot | rccl
    "mxar.engine.slot-bytes": 64 << 20,
    "mxar.engine.grid": 0,
    "mxar.engine.dtype": "bf16",
    "mxar.engine.bucket-bytes": 64 << 20,
    # GPU workers (mxar-worker --device k): the xGMI round plane (csrc/hip/xgmi_plane.h)
    "mxar.plane.dtype": "fp32",                                # fp32 | bf16 | fp16
    "mxar.plane.max-peers": 8,                                 # arena sized for <= this many workers
    "mxar.plane.max-lag": 4,                                   # ... and maxLag <= this
    "mxar.plane.grid": 0,                                      # workgroups per round launch (0: 2 per CU)
    "mxar.plane.timeout": 60.0,                                # seconds a kernel waits for a dead peer
    "mxar.plane.min-chunk": 0,                                 # one flag per chunk of >= this many elements (0: 1 KiB)
    "mxar.host-spin-us": 500,                                  # GPU worker: dispatchers / TCP readers poll this long
    "mxar.plane.spin-us": 1000,                                # completion thread polls a round this long
    "mxar.metrics.json": "",
    "mxar.trace.json": "",
}

ALIASES = {
    "akka.remote.netty.tcp.hostname": "mxar.remote.hostname",
    "akka.remote.netty.tcp.port": "mxar.remote.port",
    "akka.remote.artery.canonical.hostname": "mxar.remote.hostname",
    "akka.remote.artery.canonical.port": "mxar.remote.port",
    "akka.cluster.seed-nodes": "mxar.cluster.seed-nodes",
    "akka.cluster.roles": "mxar.cluster.roles",
    "akka.cluster.auto-down-unreachable-after": "mxar.cluster.auto-down-unreachable-after",
    "akka.cluster.failure-detector.heartbeat-interval": "mxar.cluster.failure-detector.heartbeat-interval",
    "akka.cluster.failure-detector.acceptable-heartbeat-pause":
        "mxar.cluster.failure-detector.acceptable-heartbeat-pause",
    "akka.loglevel": "mxar.loglevel",
    "akka.log-dead-letters": "mxar.log-dead-letters",
}

_DURATION = re.compile(r"^\s*([0-9]*\.?[0-9]+)\s*(ms|millis|milliseconds|s|seconds?|m|minutes?|h|hours?)\s*$")
_UNIT = {"ms": 1e-3, "millis": 1e-3, "milliseconds": 1e-3, "s": 1.0, "second": 1.0, "seconds": 1.0,
         "m": 60.0, "minute": 60.0, "minutes": 60.0, "h": 3600.0, "hour": 3600.0, "hours": 3600.0}


class ConfigError(ValueError):
    pass


# ---------------------------------------------------------------------- HOCON subset
class _Lexer:
    def __init__(self, text: str):
        self.t = text
        self.i = 0

    def skip(self, newlines: bool = True) -> None:
        while self.i < len(self.t):
            c = self.t[self.i]
            if c in " \t\r" or (newlines and c == "\n") or c == ",":
                self.i += 1
            elif c == "#" or self.t.startswith("//", self.i):
                while self.i < len(self.t) and self.t[self.i] != "\n":
                    self.i += 1
            else:
                break

    def peek(self) -> str:
        return self.t[self.i] if self.i < len(self.t) else ""

    def error(self, msg: str) -> ConfigError:
        line = self.t.count("\n", 0, self.i) + 1
        return ConfigError(f"line {line}: {msg}")


def _parse_value(lx: _Lexer) -> Any:
    lx.skip()
    c = lx.peek()
    if c == "{":
        lx.i += 1
        obj = _parse_object(lx, closing="}")
        return obj
    if c == "[":
        lx.i += 1
        items = []
        while True:
            lx.skip()
            if lx.peek() == "]":
                lx.i += 1
                return items
            if not lx.peek():
                raise lx.error("unterminated list")
            items.append(_parse_value(lx))
    if c == '"':
        j = lx.i + 1
        out = []
        while j < len(lx.t) and lx.t[j] != '"':
            if lx.t[j] == "\\" and j + 1 < len(lx.t):
                out.append({"n": "\n", "t": "\t"}.get(lx.t[j + 1], lx.t[j + 1]))
                j += 2
            else:
                out.append(lx.t[j])
                j += 1
        if j >= len(lx.t):
            raise lx.error("unterminated string")
        lx.i = j + 1
        return "".join(out)
    j = lx.i
    while j < len(lx.t) and lx.t[j] not in "\n,}]#" and not lx.t.startswith("//", j):
        if lx.t.startswith("${", j):  # substitution: ${user.dir}, ${ENV_VAR}, ${?OPTIONAL}
            k = lx.t.find("}", j)
            if k < 0:
                raise lx.error("unterminated ${")
            j = k + 1
            continue
        j += 1
    raw = lx.t[lx.i:j].strip()
    lx.i = j
    return _scalar(_substitute(raw))


_SUBST = re.compile(r"\$\{\??([A-Za-z0-9_.\-]+)\}")


def _substitute(raw: str) -> str:
    """Resolve ${user.dir} (the JVM's working directory) and ${ENV} / ${?ENV} from the
    environment; unknown references are kept verbatim."""
    def rep(m: re.Match) -> str:
        name = m.group(1)
        if name == "user.dir":
            return os.getcwd()
        return os.environ.get(name, m.group(0))

    return _SUBST.sub(rep, raw)


def _scalar(raw: str) -> Any:
    if raw in ("true", "on", "yes"):
        return True
    if raw in ("false", "off", "no"):
        return False
    if raw == "null":
        return None
    try:
        return int(raw)
    except ValueError:
        pass
    try:
        return float(raw)
    except ValueError:
        pass
    return raw


def _parse_object(lx: _Lexer, closing: str | None) -> dict:
    obj: dict = {}
    while True:
        lx.skip()
        c = lx.peek()
        if not c:
            if closing:
                raise lx.error("missing '}'")
            return obj
        if c == closing:
            lx.i += 1
            return obj
        m = re.match(r'\s*("([^"]*)"|[A-Za-z0-9_.\-]+)\s*', lx.t[lx.i:])
        if not m:
            raise lx.error(f"expected a key, found {lx.t[lx.i:lx.i + 20]!r}")
        key = m.group(2) if m.group(2) is not None else m.group(1)
        lx.i += m.end()
        c = lx.peek()
        if c in "=:":
            lx.i += 1
            val = _parse_value(lx)
        elif c == "{":
            val = _parse_value(lx)
        else:
            raise lx.error(f"expected '=', ':' or '{{' after {key!r}")
        _merge_into(obj, key.split("."), val)


def _merge_into(obj: dict, path: list[str], val: Any) -> None:
    for p in path[:-1]:
        nxt = obj.get(p)
        if not isinstance(nxt, dict):
            nxt = obj[p] = {}
        obj = nxt
    last = path[-1]
    if isinstance(val, dict) and isinstance(obj.get(last), dict):
        for k, v in val.items():
            _merge_into(obj[last], [k], v)
    else:
        obj[last] = val


def parse_hocon(text: str) -> dict:
    """Parse HOCON-subset text into a nested dict."""
    lx = _Lexer(text)
    return _parse_object(lx, closing=None)


def flatten(tree: dict, prefix: str = "") -> dict[str, Any]:
    out: dict[str, Any] = {}
    for k, v in tree.items():
        key = f"{prefix}.{k}" if prefix else k
        if isinstance(v, dict):
            out.update(flatten(v, key))
        else:
            out[key] = v
    return out


def as_seconds(v: Any) -> float:
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, str):
        if v.strip() in ("off", ""):
            return -1.0
        m = _DURATION.match(v)
        if m:
            return float(m.group(1)) * _UNIT[m.group(2)]
    raise ConfigError(f"not a duration: {v!r}")


# ---------------------------------------------------------------------- layered config
class Config:
    """Flat `mxar.*` key space with typed getters and provenance."""

    def __init__(self, values: dict[str, Any] | None = None):
        self.values: dict[str, Any] = copy.deepcopy(DEFAULTS)
        self.origin: dict[str, str] = {k: "default" for k in self.values}
        if values:
            self.update(values, "api")

    def update(self, flat: dict[str, Any], origin: str) -> "Config":
        for k, v in flat.items():
            k = ALIASES.get(k, k)
            if not k.startswith("mxar."):
                continue  # foreign keys (e.g. akka.actor.provider) are ignored, like unknown HOCON paths
            if k in ("mxar.cluster.auto-down-unreachable-after",
                     "mxar.cluster.failure-detector.heartbeat-interval",
                     "mxar.cluster.failure-detector.acceptable-heartbeat-pause"):
                v = as_seconds(v)
            self.values[k] = v
            self.origin[k] = origin
        return self

    def load_file(self, path: str) -> "Config":
        with open(path) as f:
            return self.update(flatten(parse_hocon(f.read())), path)

    def load_env(self, environ: dict[str, str] | None = None) -> "Config":
        """MXAR_ALLREDUCE_TH_REDUCE=0.5 -> mxar.allreduce.th-reduce (underscore = dot or dash
        as needed to hit a known key)."""
        environ = os.environ if environ is None else environ
        known = {k.replace(".", "_").replace("-", "_").upper(): k for k in DEFAULTS}
        flat = {}
        for name, raw in environ.items():
            if name in known:
                flat[known[name]] = _coerce(raw, DEFAULTS[known[name]])
        return self.update(flat, "env")

    def load_overrides(self, items: Iterable[str]) -> "Config":
        flat = {}
        for it in items:
            if "=" not in it:
                raise ConfigError(f"--set expects key=value, got {it!r}")
            k, v = it.split("=", 1)
            k = ALIASES.get(k.strip(), k.strip())
            flat[k] = _coerce(v.strip(), DEFAULTS.get(k))
        return self.update(flat, "cli")

    def __getitem__(self, key: str) -> Any:
        return self.values[ALIASES.get(key, key)]

    def get(self, key: str, default: Any = None) -> Any:
        return self.values.get(ALIASES.get(key, key), default)

    def set(self, key: str, value: Any, origin: str = "cli") -> None:
        self.update({key: value}, origin)

    def seeds(self) -> list[str]:
        v = self["mxar.cluster.seed-nodes"]
        return [v] if isinstance(v, str) else list(v)

    def dump(self) -> str:
        return "\n".join(f"{k} = {self.values[k]!r}  # {self.origin.get(k, '?')}" for k in sorted(self.values))


def _coerce(raw: str, like: Any) -> Any:
    if isinstance(like, bool):
        return raw.lower() in ("1", "true", "yes", "on")
    if isinstance(like, int) and not isinstance(like, bool):
        try:
            return int(raw)
        except ValueError:
            return _scalar(raw)
    if isinstance(like, float):
        try:
            return float(raw)
        except ValueError:
            return raw
    if isinstance(like, list):
        raw = raw.strip()
        if raw.startswith("["):
            return _parse_value(_Lexer(raw))
        return [x.strip() for x in raw.split(",") if x.strip()]
    return _scalar(raw)


def load(files: Iterable[str] = (), overrides: Iterable[str] = (), env: bool = True) -> Config:
    cfg = Config()
    for f in files:
        cfg.load_file(f)
    if env:
        cfg.load_env()
    cfg.load_overrides(overrides)
    return cfg
