// xorec_utils.hpp -- this repository's restatement of the part of the
// reference's src/xorec/xorec_utils.hpp that the plugin interface names
// (bm_config.hpp includes it for XorecVersion; the plugins compare codec
// statuses with XorecResult).  Same names, same values:
//   XOREC_* constants   xorec_utils.hpp:16-20
//   XorecResult         xorec_utils.hpp:26-32
//   XorecVersion        xorec_utils.hpp:38-43
// The CPU codec itself (xorec.hpp / xorec.cpp) is not part of this interface;
// its restatement is oracle/xorec_oracle.c, test infrastructure only.
//
// Used where /root/reference is absent (the GPU box, and every build of the
// product's plugin library): integration/Makefile builds the SAME plugin
// sources against the reference's own headers when they are mounted.
#ifndef XOREC_UTILS_HPP
#define XOREC_UTILS_HPP

#include <cstddef>
#include <cstdint>
#include <string>

#define XOREC_RESTRICT __restrict

constexpr size_t XOREC_BLOCK_SIZE_MULTIPLE = 256;
constexpr size_t XOREC_MIN_BLOCK_SIZE = 256;
constexpr size_t XOREC_MIN_DATA_BLOCKS = 1;
constexpr size_t XOREC_MIN_PARITY_BLOCKS = 1;
constexpr size_t XOREC_ALIGNMENT = 64;

// Status of an encode / decode (include/xec.h's xec_status 0..4 are these).
enum class XorecResult {
  Success = 0,
  InvalidSize = 1,
  InvalidAlignment = 2,
  InvalidCounts = 3,
  DecodeFailure = 4
};

// Which CPU implementation a config asks for (the GPU plugins ignore it).
enum class XorecVersion { Scalar = 0, SSE2 = 1, AVX2 = 2, AVX512 = 3 };

std::string get_version_name(XorecVersion version);

#endif  // XOREC_UTILS_HPP
