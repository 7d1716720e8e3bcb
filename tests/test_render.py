"""tablewriter v0.0.4 restatement vs README.md:294-313, on oracle verdicts (CPU only)."""
import json
import os

import numpy as np

from cyclonus_amd.probe import PlaneCells, Resources, Table, new_probe_config
from cyclonus_amd.tablewriter import render, title
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_readme_table_text_from_oracle_planes():
    c = json.load(open(os.path.join(GOLD, "config1.json")))
    status, inp, egp = O.Oracle(c["policies"], c["resources"]).probe(c["probes"])
    t = Table(Resources.from_json(c["resources"]), new_probe_config(80, "TCP"), PlaneCells(status, inp, egp), 0, 1)
    assert t.render_table() == c["readme_combined_tcp80"]["text"]


def test_title_and_multiline():
    assert title("x/a") == "X/A"
    assert title("a_b.c") == "A B C"
    out = render(["TCP/80\nTCP/81", "X/A"], [["x/a", ".\nX"]], row_line=True)
    assert out.splitlines() == [
        "+--------+-----+",
        "| TCP/80 | X/A |",
        "| TCP/81 |     |",
        "+--------+-----+",
        "| x/a    | .   |",
        "|        | X   |",
        "+--------+-----+",
    ]
