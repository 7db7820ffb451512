// peer_path_label.cpp -- integration/peer_path.hpp's labels on stubbed
// topologies (CPU only; compiled and run by tests/test_topology.py with g++).
//
//   peer_path_label pair SAME CAN LINK   -> the pair's label
//   peer_path_label scatter L1 L2 ...    -> the scatter's label over those pairs
//   peer_path_label link T               -> link_type_name(T)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "peer_path.hpp"

int main(int argc, char** argv) {
  if (argc >= 5 && std::strcmp(argv[1], "pair") == 0) {
    std::printf("%s\n", xec_hip::peer_path_label(std::atoi(argv[2]) != 0, std::atoi(argv[3]) != 0,
                                                 std::atoi(argv[4])));
    return 0;
  }
  if (argc >= 2 && std::strcmp(argv[1], "scatter") == 0) {
    std::vector<const char*> labels(argv + 2, argv + argc);
    std::printf("%s\n", xec_hip::scatter_path_label(labels.data(), labels.size()));
    return 0;
  }
  if (argc == 3 && std::strcmp(argv[1], "link") == 0) {
    std::printf("%s\n", xec_hip::link_type_name(std::atoi(argv[2])));
    return 0;
  }
  std::fprintf(stderr, "usage: peer_path_label pair SAME CAN LINK | scatter L... | link T\n");
  return 2;
}
