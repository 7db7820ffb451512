// peer_path.hpp -- names for how a root GPU's bytes reach a peer GPU (config 5's
// scatter / gather), from what the runtime reports for the pair (xec.h
// xec_peer_link).  Pure logic, no HIP: tests compile it on
// the CPU against stubbed topologies (tests/host/peer_path_label.cpp), and
// erasure-code-benchmark_amd/xec/topology.py states the same rules for
// bench.py's RCCL leg.
//
//   "local"     shard and root are the same device: a device copy;
//   "xgmi-p2p"  the device may map the peer's memory and the link is xGMI:
//               peer DMA over Infinity Fabric (SURVEY.md §8(e)'s 7 x ~153 GB/s);
//   "pcie-p2p"  peer access over PCIe;
//   "p2p"       peer access over a link of another or unreported type;
//   "staged"    no peer access: hipMemcpyPeerAsync still works, but the runtime
//               stages the bytes (through host memory), so the xGMI bound does
//               not apply and the rate is not an xGMI rate.
// A scatter over several shards is "local" when no shard is remote, "staged"
// when any remote pair is staged, the common label when all remote pairs
// agree, else "mixed".
#ifndef XEC_INTEGRATION_PEER_PATH_HPP
#define XEC_INTEGRATION_PEER_PATH_HPP

#include <cstddef>
#include <cstring>

namespace xec_hip {

// HSA link types as hipExtGetLinkTypeAndHopCount reports them
// (hsa_ext_amd.h hsa_amd_link_info_type_t)
constexpr int kLinkHyperTransport = 0, kLinkQpi = 1, kLinkPcie = 2, kLinkInfiniband = 3,
              kLinkXgmi = 4;

inline const char* link_type_name(int type) {
  switch (type) {
    case kLinkHyperTransport: return "hypertransport";
    case kLinkQpi: return "qpi";
    case kLinkPcie: return "pcie";
    case kLinkInfiniband: return "infiniband";
    case kLinkXgmi: return "xgmi";
    default: return "none";
  }
}

inline const char* peer_path_label(bool same_device, bool can_access_peer, int link_type) {
  if (same_device) return "local";
  if (!can_access_peer) return "staged";
  if (link_type == kLinkXgmi) return "xgmi-p2p";
  if (link_type == kLinkPcie) return "pcie-p2p";
  return "p2p";
}

inline const char* scatter_path_label(const char* const* labels, size_t n) {
  const char* common = nullptr;
  bool mixed = false;
  for (size_t i = 0; i < n; ++i) {
    if (std::strcmp(labels[i], "local") == 0) continue;
    if (std::strcmp(labels[i], "staged") == 0) return "staged";
    if (common == nullptr) common = labels[i];
    else if (std::strcmp(common, labels[i]) != 0) mixed = true;
  }
  if (common == nullptr) return "local";
  return mixed ? "mixed" : common;
}

}  // namespace xec_hip

#endif  // XEC_INTEGRATION_PEER_PATH_HPP
