"""Topology record of config 5's scatter, on the CPU.

The path labels are stated twice -- integration/peer_path.hpp for the C++
multi-device leg, erasure-code-benchmark_amd/xec/topology.py for bench.py's
RCCL leg -- and must agree on every stubbed pair; a pair without peer access
is "staged", never an xGMI path.  XEC_TOPOLOGY_STUB drives the record without a
GPU, and the one-GPU device list of config 5 is the repeated device 0 while a
multi-GPU node gets its distinct devices.
"""
from __future__ import annotations

import itertools
import subprocess

import pytest

from conftest import ROOT
from xec import topology
from xec.partition import config5_devices

SRC = ROOT / "tests" / "host" / "peer_path_label.cpp"


@pytest.fixture(scope="module")
def label_bin(tmp_path_factory):
    exe = tmp_path_factory.mktemp("peer_path") / "peer_path_label"
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Wextra", "-Werror",
                    f"-I{ROOT / 'integration'}", str(SRC), "-o", str(exe)], check=True)
    return exe


def _run(exe, *args):
    return subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True,
                          check=True).stdout.strip()


def test_pair_labels_agree(label_bin):
    for same, can, link in itertools.product((0, 1), (0, 1), (-1, 0, 1, 2, 3, 4, 7)):
        want = topology.peer_path_label(bool(same), bool(can), link)
        assert _run(label_bin, "pair", same, can, link) == want, (same, can, link)
    assert topology.peer_path_label(False, False, topology.LINK_XGMI) == "staged"
    assert topology.peer_path_label(False, True, topology.LINK_XGMI) == "xgmi-p2p"
    assert topology.peer_path_label(True, False, -1) == "local"


@pytest.mark.parametrize("labels,want", [
    ([], "local"), (["local"] * 8, "local"),
    (["local"] + ["xgmi-p2p"] * 7, "xgmi-p2p"),
    (["local", "xgmi-p2p", "staged", "xgmi-p2p"], "staged"),
    (["local", "xgmi-p2p", "pcie-p2p"], "mixed"),
    (["local", "pcie-p2p", "pcie-p2p"], "pcie-p2p"),
    (["staged", "staged"], "staged"),
])
def test_scatter_labels_agree(label_bin, labels, want):
    assert topology.scatter_path_label(labels) == want
    assert _run(label_bin, "scatter", *labels) == want


def test_link_names_agree(label_bin):
    for t in range(-1, 6):
        assert _run(label_bin, "link", t) == topology.link_type_name(t)


@pytest.mark.parametrize("stub,path,pair", [
    ("xgmi", "xgmi-p2p", {"can_access_peer": 1, "link_type": "xgmi", "hop_count": 1}),
    ("staged", "staged", {"can_access_peer": 0, "link_type": "none", "hop_count": None}),
    ("pcie", "pcie-p2p", {"can_access_peer": 1, "link_type": "pcie", "hop_count": 2}),
])
def test_stubbed_record(monkeypatch, stub, path, pair):
    monkeypatch.setenv("XEC_TOPOLOGY_STUB", stub)
    rec = topology.record(0, list(range(8)))
    assert rec["path"] == path and rec["root"] == 0 and "STUB" in rec["source"]
    assert rec["pairs"][0]["path"] == "local"
    for p in rec["pairs"][1:]:
        assert {k: p[k] for k in pair} == pair and p["path"] == path
    # a one-GPU list is local whatever the stub says
    assert topology.record(0, [0, 0, 0])["path"] == "local"


def test_stub_rejects_unknown(monkeypatch):
    monkeypatch.setenv("XEC_TOPOLOGY_STUB", "carrier-pigeon")
    with pytest.raises(ValueError):
        topology.record(0, [0, 1])


@pytest.mark.parametrize("visible,want", [
    (1, [0] * 8), (2, [0, 1]), (4, [0, 1, 2, 3]), (8, list(range(8))), (16, list(range(8))),
])
def test_config5_device_list(visible, want):
    assert config5_devices(visible) == want


def test_config5_device_list_needs_a_gpu():
    with pytest.raises(ValueError):
        config5_devices(0)
