// xec_multi_leg.cpp -- bench.py's "multi_device" leg: config 5 (BASELINE.json
// configs[4]: k=16+1, 1 MiB shards, stripe batches partitioned over the GPUs of
// one node) through the ONE-process multi-device plugin, XorecBenchmarkHipMulti
// (integration/xorec_hip_multi_bm.hpp, the drop-in source itself), the form
// that fits the reference's single-
// process benchmark binary.  bench.py's headline runs one process per GPU;
// this leg covers the plugin's own cross-device paths in the same run:
//
//   1. device-resident encode + decode: the reference's BM_generic iteration
//      (abstract_runner.hpp:97-121: setup | t encode | simulate_data_loss |
//      t decode | check_for_corruption) over every shard at once, timed from
//      the first launch to the last completion across the devices
//      (SURVEY.md §8(e)); losses are the reference's select_lost_blocks draw
//      (utils.cpp:100-127), and decode bytes count the data blocks actually
//      lost; every iteration's decoded batch must pass the reference's
//      validate_block check (utils.cpp:72-97) on every device;
//   2. config 5's exchange: the whole batch starts in the root device's HBM,
//      scatter_from copies each shard's stripe range to its device
//      (hipMemcpyPeerAsync over xGMI), every shard encodes, gather_parity_to
//      brings the parity back to the root, where it must equal the root's own
//      encode of the whole batch, byte for byte.
//
//   xec_multi_leg --devices 0,1,... [--stripes-per-device 256] [--data 16]
//                 [--parity 1] [--block 1M] [--iterations 10] [--warmup 3]
//                 [--root D] [--no-scatter] [--scatter-reps 3]
//
// Prints ONE JSON object on stdout; exit 0 when every check passed, 1 when a
// check failed or a call errored (the object says which), 2 on bad arguments.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "peer_path.hpp"
#include "xec.h"
#include "xec_plugin_options.hpp"
#include "xorec_hip_multi_bm.hpp"

namespace {

constexpr double kHbmPeakGBps = 8000.0;  // MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
constexpr uint64_t kSeed = 1896;         // RANDOM_SEED, utils.hpp:26

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

double median(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
}

size_t parse_size(const char* s) {
  char* end = nullptr;
  unsigned long long v = std::strtoull(s, &end, 0);
  switch (end && *end ? *end : 0) {
    case 'K': case 'k': v <<= 10; break;
    case 'M': v <<= 20; break;
    case 'G': case 'g': v <<= 30; break;
    default: break;
  }
  return static_cast<size_t>(v);
}

std::string jstr(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += (c == '\n') ? ' ' : c;
  }
  return o + "\"";
}

std::string jnum(double v, int prec = 4) {
  char b[64];
  std::snprintf(b, sizeof b, "%.*f", prec, v);
  return b;
}

using LegBench = XorecBenchmarkHipMulti;

struct Args {
  std::vector<int> devices;
  size_t S_per = 256, k = 16, m = 1, bs = 1u << 20;
  int iters = 10, warmup = 3, root = -1, scatter_reps = 3;
  bool scatter = true;
};

Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    const std::string o = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) throw std::invalid_argument(o + " needs a value");
      return argv[++i];
    };
    if (o == "--devices") {
      std::stringstream ss(val());
      std::string t;
      while (std::getline(ss, t, ',')) {
        char* end = nullptr;
        const long d = std::strtol(t.c_str(), &end, 10);
        if (t.empty() || *end || d < 0) throw std::invalid_argument("bad device " + t);
        a.devices.push_back(static_cast<int>(d));
      }
    } else if (o == "--stripes-per-device") a.S_per = parse_size(val());
    else if (o == "--data") a.k = parse_size(val());
    else if (o == "--parity") a.m = parse_size(val());
    else if (o == "--block") a.bs = parse_size(val());
    else if (o == "--iterations") a.iters = std::atoi(val());
    else if (o == "--warmup") a.warmup = std::atoi(val());
    else if (o == "--root") a.root = std::atoi(val());
    else if (o == "--scatter-reps") a.scatter_reps = std::atoi(val());
    else if (o == "--no-scatter") a.scatter = false;
    else throw std::invalid_argument("unknown option " + o);
  }
  if (a.devices.empty()) throw std::invalid_argument("--devices is required");
  if (a.iters < 1 || a.warmup < 0 || a.scatter_reps < 1 || a.S_per < 1 || a.m < 1 ||
      a.k % a.m != 0)
    throw std::invalid_argument("bad sizes or counts");
  if (a.root < 0) a.root = a.devices[0];
  return a;
}

// Config 5's exchange (scatter, per-shard encode, gather); appends its JSON
// fields to `js`, returns whether the gathered parity is bit-exact.
bool exchange(LegBench& bench, const Args& a, size_t S_total, std::string& js) {
  const size_t data_bytes = S_total * a.k * a.bs, par_bytes = S_total * a.m * a.bs;
  uint8_t *root = nullptr, *root_par = nullptr, *ref_par = nullptr;
  auto release = [&]() {
    (void)hipSetDevice(a.root);
    if (root) (void)hipFree(root);
    if (root_par) (void)hipFree(root_par);
    if (ref_par) (void)hipFree(ref_par);
  };
  if (hipSetDevice(a.root) != hipSuccess || hipMalloc(&root, data_bytes) != hipSuccess ||
      hipMalloc(&root_par, par_bytes) != hipSuccess || hipMalloc(&ref_par, par_bytes) != hipSuccess) {
    release();
    js += ",\"scatter\":{\"error\":\"root allocation failed\"}";
    return false;
  }
  // the root's batch and its own encode of it (the reference the gather must equal)
  bool ok = xec_fill_splitmix64(root, S_total, a.k * a.bs, kSeed, nullptr) == XEC_SUCCESS &&
            xec_encode(root, ref_par, S_total, a.bs, a.k, a.m, nullptr) == XEC_SUCCESS &&
            hipMemset(root_par, 0xA5, par_bytes) == hipSuccess &&
            hipDeviceSynchronize() == hipSuccess;
  std::vector<double> t_sc, t_ga;
  for (int r = 0; ok && r < a.scatter_reps; ++r) {
    const double t0 = now_s();
    ok = bench.scatter_from(root, a.root) == 0;
    t_sc.push_back(now_s() - t0);
  }
  ok = ok && bench.encode() == 0;
  for (int r = 0; ok && r < a.scatter_reps; ++r) {
    const double t0 = now_s();
    ok = bench.gather_parity_to(root_par, a.root) == 0;
    t_ga.push_back(now_s() - t0);
  }
  bool exact = false;
  if (ok) {  // compare on the host, in pieces (2 GiB of parity at 8 GPUs)
    (void)hipSetDevice(a.root);
    const size_t piece = std::min<size_t>(par_bytes, 256u << 20);
    std::vector<uint8_t> x(piece), y(piece);
    exact = true;
    for (size_t off = 0; ok && exact && off < par_bytes; off += piece) {
      const size_t n = std::min(piece, par_bytes - off);
      ok = hipMemcpy(x.data(), root_par + off, n, hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(y.data(), ref_par + off, n, hipMemcpyDeviceToHost) == hipSuccess;
      exact = ok && std::memcmp(x.data(), y.data(), n) == 0;
    }
  }
  release();
  // stripes that cross a link: every shard's range except the root's own; and
  // how each shard's copies went (peer DMA, staged by the runtime, or local)
  size_t remote = 0;
  std::vector<const char*> paths;
  std::string access = "[";
  for (size_t i = 0; i < bench.num_shards(); ++i) {
    if (bench.shard_device(i) != a.root) remote += bench.shard_count(i);
    const xec_hip::PeerAccess pa = bench.shard_peer_access(i);
    const char* name = pa == xec_hip::PeerAccess::kEnabled      ? "enabled"
                       : pa == xec_hip::PeerAccess::kStaged     ? "staged"
                       : pa == xec_hip::PeerAccess::kSameDevice ? "same-device"
                                                                : "error";
    access += std::string(i ? "," : "") + "\"" + name + "\"";
    xec_peer_link_info li{0, -1, -1};
    const bool known = xec_peer_link(bench.shard_device(i), a.root, &li) == XEC_SUCCESS;
    paths.push_back(pa == xec_hip::PeerAccess::kStaged
                        ? "staged"
                        : xec_hip::peer_path_label(bench.shard_device(i) == a.root,
                                                   known && li.can_access_peer, li.link_type));
  }
  access += "]";
  const char* path = xec_hip::scatter_path_label(paths.data(), paths.size());
  const double sc = t_sc.empty() ? 0 : *std::min_element(t_sc.begin(), t_sc.end());
  const double ga = t_ga.empty() ? 0 : *std::min_element(t_ga.begin(), t_ga.end());
  js += ",\"scatter\":{\"root\":" + std::to_string(a.root) +
        ",\"scatter_ms\":" + jnum(sc * 1e3, 3) + ",\"gather_parity_ms\":" + jnum(ga * 1e3, 3) +
        ",\"remote_stripes\":" + std::to_string(remote) +
        ",\"root_egress_GBps\":" +
        (sc > 0 ? jnum(remote * a.k * a.bs / sc / 1e9, 1) : std::string("null")) +
        ",\"root_ingress_GBps\":" +
        (ga > 0 ? jnum(remote * a.m * a.bs / ga / 1e9, 1) : std::string("null")) +
        ",\"reps\":" + std::to_string(a.scatter_reps) + ",\"path\":\"" + path + "\"" +
        ",\"peer_access_by_shard\":" + access +
        ",\"gathered_parity_bit_exact_vs_root_encode\":" + (exact ? "true" : "false") +
        (ok ? "" : ",\"error\":\"a HIP call failed during the exchange\"") +
        ",\"note\":\"batch starts in the root's HBM; hipMemcpyPeerAsync per shard: peer DMA "
        "where the pair has peer access (path xgmi-p2p over xGMI), staged by the runtime where "
        "it has not (path staged), a device copy where shard and root share one; best of "
        "reps\"}";
  return ok && exact;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  try {
    a = parse(argc, argv);
  } catch (const std::exception& e) {
    std::printf("{\"error\":%s}\n", jstr(std::string("arguments: ") + e.what()).c_str());
    return 2;
  }
  const size_t n = a.devices.size(), S_total = a.S_per * n;
  std::string js = "{\"plugin\":\"XorecBenchmarkHipMulti (one process, every device)\"";
  js += ",\"devices\":[";
  for (size_t i = 0; i < n; ++i) js += (i ? "," : "") + std::to_string(a.devices[i]);
  js += "],\"k\":" + std::to_string(a.k) + ",\"m\":" + std::to_string(a.m) +
        ",\"block_bytes\":" + std::to_string(a.bs) +
        ",\"stripes_per_device\":" + std::to_string(a.S_per) +
        ",\"stripes_total\":" + std::to_string(S_total);
  int distinct = 0;
  {
    std::vector<int> d = a.devices;
    std::sort(d.begin(), d.end());
    distinct = static_cast<int>(std::unique(d.begin(), d.end()) - d.begin());
  }
  js += ",\"distinct_devices\":" + std::to_string(distinct);
  bool pass = false;
  try {
    BenchmarkConfig c{};
    c.message_size = S_total * a.k * a.bs;
    c.block_size = a.bs;
    c.ec_params = {a.k + a.m, a.k};
    c.num_lost_blocks = 1;
    c.num_cpu_threads = 1;
    c.num_iterations = a.iters;
    c.num_warmup_iterations = a.warmup;
    c.gpu_computation = true;
    XecPluginOptions opt;
    opt.seeded = true;  // device payloads: a 32 GiB batch at 8 GPUs
    opt.seed = kSeed;
    opt.devices = a.devices;
    const double t_init = now_s();
    LegBench bench(c, opt);
    // PCI bus of each device and peer access to the root (xGMI where 1)
    js += ",\"pci_bus_ids\":[";
    for (size_t i = 0; i < n; ++i) {
      int bus = -1;
      (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, a.devices[i]);
      js += (i ? "," : "") + std::to_string(bus);
    }
    js += "],\"peer_access_to_root\":[";
    std::string topo = ",\"topology\":{\"root\":" + std::to_string(a.root) + ",\"pairs\":[";
    std::vector<const char*> labels;
    for (size_t i = 0; i < n; ++i) {
      xec_peer_link_info li{0, -1, -1};
      const bool known = xec_peer_link(a.devices[i], a.root, &li) == XEC_SUCCESS;
      const bool same = a.devices[i] == a.root;
      js += (i ? "," : "") + std::to_string(known && li.can_access_peer ? 1 : 0);
      labels.push_back(xec_hip::peer_path_label(same, known && li.can_access_peer, li.link_type));
      topo += std::string(i ? "," : "") + "{\"device\":" + std::to_string(a.devices[i]) +
              ",\"peer\":" + std::to_string(a.root) +
              ",\"can_access_peer\":" + (known ? std::to_string(li.can_access_peer) : "null") +
              ",\"link_type\":\"" + xec_hip::link_type_name(li.link_type) + "\"" +
              ",\"hop_count\":" + (li.hop_count >= 0 ? std::to_string(li.hop_count) : "null") +
              ",\"path\":\"" + labels.back() + "\"}";
    }
    js += "]" + topo + "],\"path\":\"" + xec_hip::scatter_path_label(labels.data(), labels.size()) +
          "\",\"source\":\"hipDeviceCanAccessPeer + hipExtGetLinkTypeAndHopCount (xec_peer_link)\"}";
    for (int i = 0; i < a.warmup; ++i) {
      bench.setup();
      (void)bench.encode();
      bench.simulate_data_loss();
      (void)bench.decode();
    }
    const double setup_s = now_s() - t_init;
    std::vector<double> te, td;
    size_t lost_total = 0;
    int rc = 0, corrupt = 0;
    for (int i = 0; i < a.iters; ++i) {
      bench.setup();
      const double t0 = now_s();
      rc |= bench.encode();
      const double t1 = now_s();
      bench.simulate_data_loss();
      lost_total += bench.lost_data_blocks();
      const double t2 = now_s();
      rc |= bench.decode();
      const double t3 = now_s();
      corrupt += bench.check_for_corruption() ? 0 : 1;
      te.push_back(t1 - t0);
      td.push_back(t3 - t2);
    }
    const double b_enc = double(S_total) * (a.k + a.m) * a.bs;
    const double lost_mean = double(lost_total) / a.iters;
    const double b_dec = lost_mean * (a.k / a.m + 1) * a.bs;
    const double e = median(te), d = median(td);
    const double value = (b_enc + b_dec) / (e + d) / 1e9;
    js += ",\"iterations\":" + std::to_string(a.iters) + ",\"warmup\":" + std::to_string(a.warmup) +
          ",\"encode_ms\":" + jnum(e * 1e3) + ",\"decode_ms\":" + jnum(d * 1e3) +
          ",\"encode_ms_min\":" + jnum(*std::min_element(te.begin(), te.end()) * 1e3) +
          ",\"decode_ms_min\":" + jnum(*std::min_element(td.begin(), td.end()) * 1e3) +
          ",\"encode_GBps\":" + jnum(b_enc / e / 1e9, 1) +
          ",\"decode_GBps\":" + jnum(b_dec / d / 1e9, 1) + ",\"value_GBps\":" + jnum(value, 1) +
          ",\"value_frac_of_distinct_gpu_hbm_peak\":" +
          jnum(value / (distinct * kHbmPeakGBps), 4) +
          ",\"lost_data_blocks_per_iteration\":" + jnum(lost_mean, 1) +
          ",\"codec_status\":" + std::to_string(rc) +
          ",\"corrupted_iterations\":" + std::to_string(corrupt) +
          ",\"bit_exact\":" + (rc == 0 && corrupt == 0 ? "true" : "false") +
          ",\"setup_s\":" + jnum(setup_s, 2) +
          ",\"bytes_convention\":\"algorithmic: enc S(k+m)bs + dec (lost data blocks)(k/m+1)bs; "
          "medians over iterations; wall clock first launch to last completion over the "
          "devices\"";
    pass = rc == 0 && corrupt == 0;
    if (a.scatter) pass = exchange(bench, a, S_total, js) && pass;
  } catch (const std::exception& e) {
    js += ",\"error\":" + jstr(e.what());
    pass = false;
  }
  js += "}";
  std::printf("%s\n", js.c_str());
  std::fflush(stdout);
  return pass ? 0 : 1;
}
