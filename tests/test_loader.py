"""Policy directory loader (cli/utils.go:14-60) on YAML written from the committed fixtures."""
import json
import os

import pytest
import yaml

from cyclonus_amd.loader import PolicyLoadError, read_policies_from_path

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_loads_simple_example_in_walk_order(tmp_path):
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    names = []
    for i, p in enumerate(c["policies"]):
        (tmp_path / f"{p['metadata']['name']}.yaml").write_text(json.dumps(p))
        names.append(p["metadata"]["name"])
    got = read_policies_from_path(str(tmp_path))
    assert [p["metadata"]["name"] for p in got] == [n[:-5] for n in sorted(n + ".yaml" for n in names)]
    assert sorted(json.dumps(p, sort_keys=True) for p in got) == sorted(json.dumps(p, sort_keys=True) for p in c["policies"])


def test_list_file_and_subdirs(tmp_path):
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    (tmp_path / "b").mkdir()
    (tmp_path / "b" / "list.yaml").write_text(json.dumps(c["policies"][:3]))
    (tmp_path / "a.yaml").write_text(json.dumps(c["policies"][3]))
    got = read_policies_from_path(str(tmp_path))
    assert [p["metadata"]["name"] for p in got] == [c["policies"][3]["metadata"]["name"]] + [p["metadata"]["name"] for p in c["policies"][:3]]


def test_rejects_missing_policy_types_and_unknown_fields(tmp_path):
    (tmp_path / "x.yaml").write_text("kind: NetworkPolicy\nmetadata: {name: a, namespace: b}\nspec: {podSelector: {}}\n")
    with pytest.raises(PolicyLoadError, match="missing spec.policyTypes from network policy b/a"):
        read_policies_from_path(str(tmp_path))
    (tmp_path / "x.yaml").write_text("kind: NetworkPolicy\nbogus: 1\nspec: {podSelector: {}, policyTypes: [Ingress]}\n")
    with pytest.raises(PolicyLoadError, match="unable to unmarshal"):
        read_policies_from_path(str(tmp_path))


def _one(tmp_path, text):
    (tmp_path / "x.yaml").write_text(text)
    return read_policies_from_path(str(tmp_path))


POL = "kind: NetworkPolicy\nmetadata: {name: a, namespace: %s}\nspec: {podSelector: {}, policyTypes: [Ingress]}\n"


def test_yaml11_scalars_coerced_into_string_fields(tmp_path):
    """sigs.k8s.io/yaml v1.2.0 convertToJSONableObject: YAML 1.1 bools / ints / floats landing in Go
    string fields become their text (parity unpinned: no reference fixture has them unquoted)."""
    for raw, want in (("y", "true"), ("Yes", "true"), ("off", "false"), ("010", "8"), ("0x1F", "31"), ("1_000", "1000"),
                      ("1.5", "1.5"), ("1e6", "1e+06"), ("100000.0", "100000"), ("0.1", "0.1"), ("2001-12-14", "2001-12-14"),
                      ("'y'", "y"), ("x-y", "x-y")):
        got = _one(tmp_path, POL % raw)
        assert got[0]["metadata"]["namespace"] == want, raw
    got = _one(tmp_path, "kind: NetworkPolicy\nmetadata: {name: a, labels: {y: on, 7: 2.50}}\n"
                         "spec: {podSelector: {matchLabels: {n: 3}}, policyTypes: [Ingress],"
                         " ingress: [{ports: [{port: 80}, {port: '81', protocol: UDP}]}]}\n")
    assert got[0]["metadata"]["labels"] == {"true": "true", "7": "2.5"}
    assert got[0]["spec"]["podSelector"]["matchLabels"] == {"false": "3"}
    assert got[0]["spec"]["ingress"][0]["ports"] == [{"port": 80}, {"port": "81", "protocol": "UDP"}]  # intstr: no coercion


def test_first_document_only_and_strictness(tmp_path):
    two = POL % "one" + "---\n" + POL % "two"
    assert [p["metadata"]["namespace"] for p in _one(tmp_path, two)] == ["one"]
    # UnmarshalStrict: unknown fields at any depth and duplicate keys are errors for a single policy...
    for bad in ("kind: NetworkPolicy\nspec: {podSelectr: {}, policyTypes: [Ingress]}\n",
                "kind: NetworkPolicy\nstatus: {}\nspec: {policyTypes: [Ingress]}\n",
                "kind: NetworkPolicy\nkind: NetworkPolicy\nspec: {policyTypes: [Ingress]}\n",
                "kind: NetworkPolicy\nspec: {policyTypes: Ingress}\n"):
        with pytest.raises(PolicyLoadError, match="unable to unmarshal single policy"):
            _one(tmp_path, bad)
    # ...while the list form (yaml.Unmarshal) drops unknown fields and lets a later key win
    got = _one(tmp_path, "- kind: NetworkPolicy\n  metadata: {name: a, name: b}\n"
                         "  spec: {podSelectr: {}, policyTypes: [Egress]}\n")
    assert got == [{"kind": "NetworkPolicy", "metadata": {"name": "b"}, "spec": {"policyTypes": ["Egress"]}}]
    # field names match case-insensitively; the last key naming a field wins
    got = _one(tmp_path, "Kind: NetworkPolicy\nMetadata: {Name: a, namespace: p, Namespace: q}\nSPEC: {policyTypes: [Ingress]}\n")
    assert got[0]["metadata"] == {"name": "a", "namespace": "q"} and got[0]["kind"] == "NetworkPolicy"
    assert _one(tmp_path, "") == []  # an empty file is an empty list


YAML = os.path.join(GOLD, "yaml")


def test_reference_policy_files():
    """The reference's own policy files (networkpolicies/**, copied byte for byte by
    tests/golden/make_fixtures.py): plain scalars (`pod: b`, `values: [a, b]`), a commented-out line,
    multi-rule lists.  The simple-example directory loads to config #1's policies in filepath.Walk
    order, and each fixture file to its policies."""
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    got = read_policies_from_path(os.path.join(YAML, "simple-example"))
    assert json.dumps(got, sort_keys=True) == json.dumps(c["policies"], sort_keys=True)
    fx = json.load(open(os.path.join(GOLD, "policy_fixtures.json")))
    for rel, want in fx.items():
        path = os.path.join(YAML, os.path.relpath(rel, "networkpolicies"))
        assert json.dumps(read_policies_from_path(path), sort_keys=True) == json.dumps(want, sort_keys=True), rel
    # the whole tree: every file, directories descended in lexical order
    every = read_policies_from_path(YAML)
    assert len(every) == len(c["policies"]) + sum(len(v) for v in fx.values())
