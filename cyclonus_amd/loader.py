"""Policy directory loader: restates cli/utils.go:14-60 readPoliciesFromPath.

Walk the path in lexical order (filepath.Walk); parse each file first as a list of NetworkPolicies
(sigs.k8s.io/yaml Unmarshal), else as one policy (UnmarshalStrict); reject policies with an empty
spec.policyTypes.

sigs.k8s.io/yaml v1.2.0 is not vendored in the reference (go.mod / go.sum only), so its published
algorithm is restated here:

* YAML -> generic tree with gopkg.in/yaml.v2 (YAML 1.1): ONLY THE FIRST DOCUMENT of a file is
  decoded; plain scalars resolve as go-yaml v2's resolve() does (`y`/`Yes`/`on`/... are booleans,
  `0x1F`, `010` (octal), `1_000` are ints, `1.5`/`.5`/`.inf` floats, `~`/`null`/empty are null,
  timestamp-like scalars stay strings); quoted scalars are always strings.  Strict mode rejects
  duplicate mapping keys.
* convertToJSONableObject walks the tree WITH THE TARGET TYPE: a bool / int / float landing in a
  Go string field (or map[string]string value, or []string element) becomes its text — "true" /
  "false", decimal ints, floats by strconv.FormatFloat(v, 'g', -1, 32); mapping keys become strings
  the same way.  Types with their own UnmarshalJSON (intstr.IntOrString for `port`, metav1.Time)
  are passed through unconverted.
* encoding/json decodes that into *networkingv1.NetworkPolicy (k8s.io/api v0.21.0-rc.0): struct
  fields match exactly or ASCII case-insensitively (the last matching key wins); wrong JSON types
  are errors; unknown fields are dropped by Unmarshal and are errors at ANY depth under
  UnmarshalStrict (DisallowUnknownFields).

Parity unpinned: the reference holds no fixture with unquoted non-string scalars, duplicate keys,
multi-document files or unknown nested fields (its own YAML quotes `"y"`, networkpolicies/); these
rules follow the published library sources cited above.
"""
from __future__ import annotations

import math
import os
import re
from typing import Any

import numpy as np
import yaml

__all__ = ["PolicyLoadError", "read_policies_from_path", "load_policies_yaml"]


class PolicyLoadError(ValueError):
    pass


class _Fail(Exception):
    pass


# ----------------------------------------------------------------------------- YAML 1.1 scalars
class _PlainLoader(yaml.SafeLoader):
    """Composer only: no implicit resolvers, so plain scalars keep their text (resolved below)."""


_PlainLoader.yaml_implicit_resolvers = {}

_BOOL = {**{s: True for s in ("y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON")},
         **{s: False for s in ("n", "N", "no", "No", "NO", "false", "False", "FALSE", "off", "Off", "OFF")}}
_NULL = {"", "~", "null", "Null", "NULL"}
_SPECIAL_FLOAT = {**{s: math.nan for s in (".nan", ".NaN", ".NAN")},
                  **{s: math.inf for s in (".inf", ".Inf", ".INF", "+.inf", "+.Inf", "+.INF")},
                  **{s: -math.inf for s in ("-.inf", "-.Inf", "-.INF")}}
_YAML_FLOAT = re.compile(r"^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$")  # go-yaml yamlStyleFloat
_GO_INT = re.compile(r"^[-+]?(0[xX][0-9a-fA-F]+|0[oO][0-7]+|0[bB][01]+|0[0-7]*|[1-9][0-9]*)$")  # ParseInt(s, 0, 64)
_TIMESTAMP = [re.compile(p) for p in (  # go-yaml allowedTimestampFormats
    r"^\d{4}-\d{1,2}-\d{1,2}([Tt]|\s+)\d{1,2}:\d{2}:\d{2}(\.\d+)?(\s*([Zz]|[-+]\d{1,2}(:\d{2})?))?$",
    r"^\d{4}-\d{2}-\d{2}$")]


def _go_parse_int(s: str):
    if not _GO_INT.match(s):
        return None
    sign, body = (-1, s[1:]) if s[0] == "-" else (1, s[1:] if s[0] == "+" else s)
    if body[:2] in ("0x", "0X"):
        v = int(body[2:], 16)
    elif body[:2] in ("0o", "0O"):
        v = int(body[2:], 8)
    elif body[:2] in ("0b", "0B"):
        v = int(body[2:], 2)
    elif len(body) > 1 and body[0] == "0":
        v = int(body[1:], 8)
    else:
        v = int(body)
    v *= sign
    if -(1 << 63) <= v < (1 << 63) or (sign > 0 and v < (1 << 64)):  # ParseInt, then ParseUint
        return v
    return None


def _resolve_plain(s: str) -> Any:
    """go-yaml v2 resolve() for an untagged plain scalar (resolve.go), timestamps kept as text."""
    if s in _NULL:
        return None
    if s in _BOOL:
        return _BOOL[s]
    if s in _SPECIAL_FLOAT:
        return _SPECIAL_FLOAT[s]
    c = s[0]
    if c == ".":
        try:
            return float(s) if re.match(r"^\.[0-9]+([eE][-+]?[0-9]+)?$", s) else s
        except ValueError:
            return s
    if c in "+-0123456789":
        if any(p.match(s) for p in _TIMESTAMP):
            return s  # decoded into interface{} as the string (backward compatibility in v2)
        plain = s.replace("_", "")
        v = _go_parse_int(plain)
        if v is not None:
            return v
        if _YAML_FLOAT.match(plain):
            return float(plain)
        for pre, sign in (("0b", 1), ("-0b", -1)):
            if plain.startswith(pre) and re.match(r"^[01]+$", plain[len(pre):]):
                return sign * int(plain[len(pre):], 2)
    return s


class _Map(list):
    """A decoded YAML mapping: [(key, value)] in document order."""


def _tree(node, strict: bool):
    """PyYAML node -> generic value as go-yaml v2 decodes into interface{}."""
    if node is None:
        return None
    if isinstance(node, yaml.ScalarNode):
        if node.tag == "tag:yaml.org,2002:str" and node.style is None:
            return _resolve_plain(node.value)
        if node.tag in ("tag:yaml.org,2002:int", "tag:yaml.org,2002:float", "tag:yaml.org,2002:bool",
                        "tag:yaml.org,2002:null"):
            return _resolve_plain(node.value)
        return node.value
    if isinstance(node, yaml.SequenceNode):
        return [_tree(n, strict) for n in node.value]
    out, keys = {}, set()
    for kn, vn in node.value:
        k = _tree(kn, strict)
        hk = ("b", k) if isinstance(k, bool) else ("v", k)
        if strict and hk in keys:  # yaml.UnmarshalStrict: duplicate mapping keys are errors
            raise _Fail(f"mapping key {k!r} already defined")
        keys.add(hk)
        out[hk] = (k, _tree(vn, strict))
    return _Map(out.values())  # [(key, value)] in document order (a later duplicate overwrote)


def _first_document(text: str, strict: bool):
    loader = _PlainLoader(text)
    try:
        node = loader.get_node() if loader.check_node() else None  # the first document only
    except yaml.YAMLError as e:
        raise _Fail(str(e))
    finally:
        loader.dispose()
    return _tree(node, strict)


# ----------------------------------------------------------------------------- target types
def _go_float32_g(v: float) -> str:
    """strconv.FormatFloat(v, 'g', -1, 32)."""
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    f = np.float32(v)
    if f == 0:
        return "-0" if math.copysign(1.0, float(f)) < 0 else "0"
    sci = np.format_float_scientific(f, unique=True, trim="-")  # shortest float32 digits
    mant, exp = sci.split("e")
    neg = mant.startswith("-")
    digits = mant.lstrip("-").replace(".", "")
    e = int(exp)
    if e < -4 or e >= 6:  # %e when the exponent < -4 or >= eprec (6 for the shortest form)
        m = digits[0] + ("." + digits[1:] if len(digits) > 1 else "")
        s = f"{m}e{'-' if e < 0 else '+'}{abs(e):02d}"
    elif e >= 0:
        s = digits[: e + 1].ljust(e + 1, "0") + ("." + digits[e + 1:] if len(digits) > e + 1 else "")
    else:
        s = "0." + "0" * (-e - 1) + digits
    return ("-" if neg else "") + s


def _key_string(k) -> str:
    if isinstance(k, bool):
        return "true" if k else "false"
    if isinstance(k, int):
        return str(k)
    if isinstance(k, float):
        s = _go_float32_g(k)
        return {"+Inf": ".inf", "-Inf": "-.inf", "NaN": ".nan"}.get(s, s)
    if isinstance(k, str):
        return k
    raise _Fail(f"Unsupported map key of type {type(k).__name__}")


# Go field types: STR / INT are plain fields, PSTR / PINT / INTSTR pointers (*Protocol, *int32,
# *intstr.IntOrString): a JSON null sets a pointer to nil and leaves a plain field as it was
STR, PSTR, INT, PINT, BOOL, INTSTR, ANY = "string", "*string", "int", "*int", "bool", "intstr", "any"


def _map(t):
    return ("map", t)


def _list(t):
    return ("list", t)


_SELECTOR = {"matchLabels": _map(STR),
             "matchExpressions": _list({"key": STR, "operator": STR, "values": _list(STR)})}
_PORT = {"protocol": PSTR, "port": INTSTR, "endPort": PINT}
_PEER = {"podSelector": _SELECTOR, "namespaceSelector": _SELECTOR, "ipBlock": {"cidr": STR, "except": _list(STR)}}
_OWNER = {"apiVersion": STR, "kind": STR, "name": STR, "uid": STR, "controller": BOOL, "blockOwnerDeletion": BOOL}
_MANAGED = {"manager": STR, "operation": STR, "apiVersion": STR, "time": ANY, "fieldsType": STR, "fieldsV1": ANY}
_META = {"name": STR, "generateName": STR, "namespace": STR, "selfLink": STR, "uid": STR, "resourceVersion": STR,
         "generation": INT, "creationTimestamp": ANY, "deletionTimestamp": ANY, "deletionGracePeriodSeconds": PINT,
         "labels": _map(STR), "annotations": _map(STR), "ownerReferences": _list(_OWNER), "finalizers": _list(STR),
         "clusterName": STR, "managedFields": _list(_MANAGED)}
# networking.k8s.io/v1 NetworkPolicy at k8s.io/api v0.21.0-rc.0 (TypeMeta inline, ObjectMeta, Spec)
NETWORK_POLICY = {"kind": STR, "apiVersion": STR, "metadata": _META,
                  "spec": {"podSelector": _SELECTOR,
                           "ingress": _list({"ports": _list(_PORT), "from": _list(_PEER)}),
                           "egress": _list({"ports": _list(_PORT), "to": _list(_PEER)}),
                           "policyTypes": _list(STR)}}


def _convert(v, t, strict: bool, path: str):
    """convertToJSONableObject + encoding/json into the target type (errors raise _Fail)."""
    if v is None:
        return None  # JSON null: nil for maps / slices / pointers, no effect otherwise
    if t == ANY:
        return _plain_json(v)
    if isinstance(t, dict) or (isinstance(t, tuple) and t[0] == "map"):
        if not isinstance(v, _Map):
            raise _Fail(f"{path}: cannot unmarshal {_kind(v)} into an object")
        out = {}
        for k, x in v:
            ks = _key_string(k)
            if isinstance(t, tuple):  # map[string]T
                out[ks] = _convert(x, t[1], strict, f"{path}.{ks}")
                continue
            f = ks if ks in t else next((n for n in t if n.lower() == ks.lower()), None)
            if f is None:
                if strict:  # DisallowUnknownFields, at every depth
                    raise _Fail(f'{path}: unknown field "{ks}"')
                continue
            val = _convert(x, t[f], strict, f"{path}.{f}")
            if val is None and f in out and t[f] in (STR, INT, BOOL):
                continue  # null into a plain (non-pointer) field leaves the earlier value
            out[f] = val  # several keys folding onto one field: the last one wins
        return out
    if isinstance(t, tuple) and t[0] == "list":
        if isinstance(v, _Map) or not isinstance(v, list):
            raise _Fail(f"{path}: cannot unmarshal {_kind(v)} into an array")
        return [_convert(x, t[1], strict, f"{path}[{i}]") for i, x in enumerate(v)]
    if t in (STR, PSTR):
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, int):
            return str(v)
        if isinstance(v, float):
            return _go_float32_g(v)
        if isinstance(v, str):
            return v
        raise _Fail(f"{path}: cannot unmarshal {_kind(v)} into a string")
    if t == BOOL:
        if isinstance(v, bool):
            return v
        raise _Fail(f"{path}: cannot unmarshal {_kind(v)} into a bool")
    if t in (INT, PINT, INTSTR):
        if isinstance(v, bool):
            raise _Fail(f"{path}: cannot unmarshal bool into a number")
        if isinstance(v, int):
            return v
        if isinstance(v, float) and math.isfinite(v) and v == int(v) and abs(v) < 1e21:
            return int(v)  # json.Marshal(float64(80)) is 80
        if t == INTSTR and isinstance(v, str):
            return v
        raise _Fail(f"{path}: cannot unmarshal {_kind(v)} into an integer")
    raise AssertionError(t)


def _kind(v):
    return {bool: "bool", int: "number", float: "number", str: "string"}.get(type(v), "object" if isinstance(v, _Map) else "array")


def _plain_json(v):
    if isinstance(v, _Map):
        return {_key_string(k): _plain_json(x) for k, x in v}
    if isinstance(v, list):
        return [_plain_json(x) for x in v]
    return v


# ----------------------------------------------------------------------------- the reader
def load_policies_yaml(text: str, path: str = "<input>"):
    """One file's policies, as readPoliciesFromPath's per-file callback (utils.go:24-49)."""
    try:  # try parsing a list first (utils.go:30-37): yaml.Unmarshal into []*NetworkPolicy
        doc = _first_document(text, strict=False)
        if doc is None:
            return []
        if isinstance(doc, list) and not isinstance(doc, _Map):
            pols = _convert(doc, _list(NETWORK_POLICY), False, "")
            if any(p is None for p in pols):
                raise PolicyLoadError(f"nil policy in the list at {path} (the reference dereferences it)")
            return pols
    except _Fail:
        pass
    try:  # single policy (utils.go:39-45): yaml.UnmarshalStrict into *NetworkPolicy
        doc = _first_document(text, strict=True)
        if doc is None:
            raise PolicyLoadError(f"nil policy at {path} (the reference dereferences it)")
        return [_convert(doc, NETWORK_POLICY, True, "")]
    except _Fail as e:
        raise PolicyLoadError(f"unable to unmarshal single policy from yaml at {path}: {e}")


def read_policies_from_path(policy_path: str):
    files = []
    if os.path.isfile(policy_path):
        files = [policy_path]
    else:  # filepath.Walk: lexical order, directories descended in place
        for root, dirs, names in os.walk(policy_path):
            dirs.sort()
            for n in sorted(names):
                files.append(os.path.join(root, n))
        files.sort(key=lambda f: os.path.relpath(f, policy_path).split(os.sep))
    policies = []
    for f in files:
        with open(f, encoding="utf-8", errors="surrogateescape") as fh:
            policies += load_policies_yaml(fh.read(), f)
    for p in policies:  # utils.go:54-58
        spec = p.get("spec") or {}
        if not spec.get("policyTypes"):
            md = p.get("metadata") or {}
            raise PolicyLoadError(f"missing spec.policyTypes from network policy {md.get('namespace') or ''}/{md.get('name') or ''}")
    return policies
