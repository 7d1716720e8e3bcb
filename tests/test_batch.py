"""Host side of the batched-blocks mode (cyclonus_amd/batch.py, no GPU): every block's namespaces are
renamed "<block>~<ns>" exactly as the library's loader would decode them (encoding/json: fields match
case-insensitively, the last non-null key wins, a null is absent)."""
from cyclonus_amd.batch import Batch


def _pod(**kw):
    p = {"Name": "a", "Labels": {"app": "a"}, "IP": "10.0.0.1",
         "Containers": [{"Name": "c", "Port": 80, "Protocol": "TCP", "PortName": "serve-80-tcp"}]}
    p.update(kw)
    return p


def _policy(metadata):
    return {"metadata": metadata, "spec": {"podSelector": {}, "policyTypes": ["Ingress"]}}


def test_block_namespaces_follow_the_loader():
    probe = {"Port": 80, "Protocol": "TCP"}
    pods = [
        _pod(Namespace="x"),
        _pod(namespace="x"),                      # lowercase key: still the Namespace field
        _pod(Namespace="x", namespace=None),      # a later null leaves "x"
        _pod(Namespace=None),                     # null: absent -> ""
        _pod(),                                   # absent
        _pod(Namespace="y", NAMESPACE="x"),       # the last matching key wins
    ]
    pols = [
        _policy({"name": "p0", "namespace": "x"}),
        _policy({"name": "p1", "Namespace": "x"}),
        _policy({"name": "p2", "namespace": None}),
        _policy(None),
        {"Metadata": {"name": "p4", "namespace": "x"}, "spec": {"podSelector": {}, "policyTypes": ["Ingress"]}},
        {"spec": {"podSelector": {}, "policyTypes": ["Ingress"]}},
    ]
    bt = Batch([{"policies": pols, "resources": {"Namespaces": {"x": {}}, "Pods": pods}, "probe": probe}] * 2)
    got_pods = [[k for k in p if k.lower() == "namespace"] for p in bt.resources["Pods"]]
    assert all(keys == ["Namespace"] for keys in got_pods)
    assert [p["Namespace"] for p in bt.resources["Pods"][:6]] == ["0~x", "0~x", "0~x", "0~", "0~", "0~x"]
    assert [p["Namespace"] for p in bt.resources["Pods"][6:]] == ["1~x", "1~x", "1~x", "1~", "1~", "1~x"]
    mds = [p["metadata"] for p in bt.policies]
    assert all([k for k in p if k.lower() == "metadata"] == ["metadata"] for p in bt.policies)
    assert [m["namespace"] for m in mds[:6]] == ["0~x", "0~x", "0~default", "0~default", "0~x", "0~default"]
    assert [m["namespace"] for m in mds[6:]] == ["1~x", "1~x", "1~default", "1~default", "1~x", "1~default"]
    assert sorted(bt.resources["Namespaces"]) == ["0~x", "1~x"]
