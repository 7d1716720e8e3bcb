"""Policy directory loader: restates cli/utils.go:14-60 readPoliciesFromPath.

Walk the path in lexical order (filepath.Walk), parse each file first as a YAML list of
NetworkPolicies, else as one policy (strict: unknown top-level fields rejected, as
yaml.UnmarshalStrict does), and reject policies with an empty spec.policyTypes.  YAML is read as
sigs.k8s.io/yaml v1.2.0 (go-yaml v2, YAML 1.1) reads it: y / Y / n / N are booleans too.
"""
from __future__ import annotations

import os
import re

import yaml


class _Go11Loader(yaml.SafeLoader):
    pass


_Go11Loader.add_implicit_resolver(
    "tag:yaml.org,2002:bool",
    re.compile(r"^(?:y|Y|yes|Yes|YES|n|N|no|No|NO|true|True|TRUE|false|False|FALSE|on|On|ON|off|Off|OFF)$"),
    list("yYnNtTfFoO"),
)
_BOOL = {"y": True, "yes": True, "true": True, "on": True, "n": False, "no": False, "false": False, "off": False}
_Go11Loader.add_constructor("tag:yaml.org,2002:bool", lambda loader, node: _BOOL[loader.construct_scalar(node).lower()])

_TOP = {"apiVersion", "kind", "metadata", "spec", "status"}


class PolicyLoadError(ValueError):
    pass


def _check_types(p, path):
    if not isinstance(p, dict):
        raise PolicyLoadError(f"unable to unmarshal single policy from yaml at {path}")
    for key in ("metadata", "spec"):
        if key in p and p[key] is not None and not isinstance(p[key], dict):
            raise PolicyLoadError(f"unable to unmarshal single policy from yaml at {path}")
    md = p.get("metadata") or {}
    for k in ("name", "namespace"):
        if k in md and not isinstance(md[k], str):
            raise PolicyLoadError(f"unable to unmarshal single policy from yaml at {path}: {k} is not a string")


def read_policies_from_path(policy_path: str):
    files = []
    if os.path.isfile(policy_path):
        files = [policy_path]
    else:
        for root, dirs, names in os.walk(policy_path):
            dirs.sort()
            for n in sorted(names):
                files.append(os.path.join(root, n))
        files.sort(key=lambda f: os.path.relpath(f, policy_path).split(os.sep))
    policies = []
    for f in files:
        with open(f) as fh:
            doc = yaml.load(fh, Loader=_Go11Loader)
        if doc is None or isinstance(doc, list):  # list first (utils.go:31-37)
            for p in doc or []:
                _check_types(p, f)
            policies += list(doc or [])
            continue
        if not isinstance(doc, dict) or set(doc) - _TOP:  # UnmarshalStrict (utils.go:40-45)
            raise PolicyLoadError(f"unable to unmarshal single policy from yaml at {f}")
        _check_types(doc, f)
        policies.append(doc)
    for p in policies:  # utils.go:54-58
        spec = p.get("spec") or {}
        if not spec.get("policyTypes"):
            md = p.get("metadata") or {}
            raise PolicyLoadError(f"missing spec.policyTypes from network policy {md.get('namespace', '')}/{md.get('name', '')}")
    return policies
