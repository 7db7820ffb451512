"""How config 5's scatter reaches each peer GPU.

The N > 1 runs move stripe ranges from a root GPU to its peers: RCCL send /
recv between ranks (xec/dist.py) and hipMemcpyPeerAsync in the one-process
plugin (integration/xorec_hip_multi_bm.cpp).  Whether those bytes go by peer
DMA over xGMI -- the link SURVEY.md §8(e) bounds at 7 x ~153 GB/s per GPU --
or are staged by the runtime depends on the pair, so every N > 1 line records,
per root -> peer pair, what the runtime reports (include/xec.h xec_peer_link:
hipDeviceCanAccessPeer + hipExtGetLinkTypeAndHopCount) and labels the path.
The labels follow integration/peer_path.hpp (the C++ leg's), rule for rule;
tests/test_topology.py checks the two agree on stubbed topologies.

XEC_TOPOLOGY_STUB (tests and CPU rehearsals only) replaces the runtime query:
"xgmi" -- every distinct pair peer-accessible over one xGMI hop; "staged" --
no pair peer-accessible; "pcie" -- peer access over PCIe, two hops.
"""
from __future__ import annotations

import ctypes
import os

LINK_NAMES = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}
LINK_PCIE, LINK_XGMI = 2, 4

_STUBS = {"xgmi": (1, LINK_XGMI, 1), "staged": (0, -1, -1), "pcie": (1, LINK_PCIE, 2)}


def link_type_name(t: int) -> str:
    return LINK_NAMES.get(t, "none")


def peer_path_label(same_device: bool, can_access_peer: bool, link_type: int) -> str:
    """peer_path.hpp peer_path_label."""
    if same_device:
        return "local"
    if not can_access_peer:
        return "staged"
    if link_type == LINK_XGMI:
        return "xgmi-p2p"
    if link_type == LINK_PCIE:
        return "pcie-p2p"
    return "p2p"


def scatter_path_label(labels) -> str:
    """peer_path.hpp scatter_path_label: "local" with no remote pair, "staged"
    if any remote pair is staged, the common label, else "mixed"."""
    remote = [x for x in labels if x != "local"]
    if not remote:
        return "local"
    if "staged" in remote:
        return "staged"
    return remote[0] if len(set(remote)) == 1 else "mixed"


class _PeerLink(ctypes.Structure):
    _fields_ = [("can_access_peer", ctypes.c_int), ("link_type", ctypes.c_int),
                ("hop_count", ctypes.c_int)]


def _query(device: int, peer: int):
    """(can_access_peer, link_type, hop_count) from the runtime, or from
    XEC_TOPOLOGY_STUB."""
    stub = os.environ.get("XEC_TOPOLOGY_STUB", "").strip().lower()
    if stub:
        if device == peer:
            return 1, -1, -1
        if stub not in _STUBS:
            raise ValueError(f"XEC_TOPOLOGY_STUB={stub!r}: one of {sorted(_STUBS)}")
        return _STUBS[stub]
    from ._lib import lib
    info = _PeerLink()
    st = lib().xec_peer_link(int(device), int(peer), ctypes.byref(info))
    if st != 0:
        raise RuntimeError(f"xec_peer_link({device}, {peer}) returned {st}")
    return info.can_access_peer, info.link_type, info.hop_count


def record(root: int, devices) -> dict:
    """The topology record of a scatter from `root` to `devices` (one entry per
    device, repeats allowed): per pair the runtime's answers and the path
    label, and the scatter's overall path."""
    pairs = []
    for d in devices:
        can, lt, hops = _query(d, root)
        pairs.append({"device": int(d), "peer": int(root), "can_access_peer": int(can),
                      "link_type": link_type_name(lt), "hop_count": hops if hops >= 0 else None,
                      "path": peer_path_label(d == root, bool(can), lt)})
    out = {"root": int(root), "pairs": pairs,
           "path": scatter_path_label([p["path"] for p in pairs]),
           "source": "hipDeviceCanAccessPeer + hipExtGetLinkTypeAndHopCount (xec_peer_link)"}
    if os.environ.get("XEC_TOPOLOGY_STUB"):
        out["source"] = f"STUB XEC_TOPOLOGY_STUB={os.environ['XEC_TOPOLOGY_STUB']} (not measured)"
    return out
