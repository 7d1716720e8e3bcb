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


def test_yaml11_booleans_like_go_yaml_v2(tmp_path):
    # an unquoted `namespace: y` is a boolean for go-yaml v2, so the reference cannot load it
    (tmp_path / "x.yaml").write_text("kind: NetworkPolicy\nmetadata: {name: a, namespace: y}\nspec: {podSelector: {}, policyTypes: [Ingress]}\n")
    with pytest.raises(PolicyLoadError):
        read_policies_from_path(str(tmp_path))
