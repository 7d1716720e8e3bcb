"""Config #5 generator restatement: case / step counts pinned by
pkg/generator/testcasegenerator_tests.go:92-108 and SURVEY.md §8d."""
from cyclonus_amd import generator as g


def test_case_counts():
    gen = g.Generator("192.168.1.9")
    assert len(gen.target_cases()) == 6
    assert len(gen.rules_cases()) == 4
    assert len(gen.peers_cases()) == 112
    assert len(gen.port_protocol_cases()) == 58
    assert len(gen.example_cases()) == 1
    assert len(gen.action_cases()) == 6
    assert len(gen.conflict_cases()) == 16
    assert len(gen.upstream_cases()) == 13
    assert len(gen.all_cases()) == 216


def test_sweep_steps_and_mock_ips():
    steps = g.sweep()
    assert len(steps) == 242
    zc = [p for p in steps[0]["resources"]["Pods"] if p["Namespace"] == "z" and p["Name"] == "c"][0]
    assert zc["IP"] == "192.168.1.9"
    created = [p["IP"] for s in steps for p in s["resources"]["Pods"] if (p["Namespace"], p["Name"]) in {("w", "a"), ("y-2", "a"), ("y-2", "b"), ("x", "d")}]
    assert set(created) == {"192.168.1.10", "192.168.1.11", "192.168.1.12", "192.168.1.13"}
    # ipBlock peers are built from z/c's IP (peerscases.go:15-21)
    cidrs = {str(pe.get("ipBlock", {}).get("cidr")) for s in steps for pol in s["policies"] for r in pol["spec"].get("ingress", []) for pe in r.get("from", [])}
    assert "192.168.1.0/24" in cidrs


def test_batch_layout():
    from cyclonus_amd.batch import Batch

    steps = g.sweep()[:5]
    bt = Batch(steps)
    assert len(bt.resources["Pods"]) == sum(len(s["resources"]["Pods"]) for s in steps)
    assert all(p["metadata"]["namespace"].split("~")[0].isdigit() for p in bt.policies)
