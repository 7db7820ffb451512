// ref_iface_prelude.hpp -- force-included (-include) when the plugin is compiled
// against the reference's unmodified headers (integration/Makefile).
//
// The reference's bm_config.hpp includes console_reporter.hpp, which includes
// Google Benchmark (<benchmark/benchmark.h>); the library is an empty git
// submodule in the reference (libraries/google_benchmark) and absent from this
// image.  bm_config.hpp names only two of its types, and only as incomplete
// types: `ConsoleReporter* reporter` (bm_config.hpp:42) and the parameter
// `benchmark::State&` of the BenchmarkFunction pointer type (:48).  The build
// defines CONSOLE_REPORTER_HPP (console_reporter.hpp's include guard) and
// declares those two names here; nothing is defined, and no code path of the
// plugin, abstract_bm.cpp or utils.cpp uses either type.  bm_config.hpp also
// relies on benchmark.h for <tuple> (ECTuple, :18), so that standard header is
// included here.
#ifndef XEC_REF_IFACE_PRELUDE_HPP
#define XEC_REF_IFACE_PRELUDE_HPP

#include <tuple>

namespace benchmark {
class State;
}
class ConsoleReporter;

#endif  // XEC_REF_IFACE_PRELUDE_HPP
