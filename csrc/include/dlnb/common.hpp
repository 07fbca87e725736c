// Common definitions for the dlnb native runtime: error handling, element
// types and small string helpers.
//
// Parity notes (reference = HicrestLaboratory/DLNetBench):
//   * The reference selects element/wire types with compile-time macros
//     (cpp/data_types.hpp:36-79) and ends up allocating 4-byte floats while
//     putting bf16 on the CCL wire. Here the element type IS the wire type and
//     is chosen at run time (DType below); buffers are sized exactly.
//   * Error checks replace ccutils' CUDA macros / cpp/tmp_hip_ccutils.hpp:6-19
//     with exceptions that carry file:line, so a failing rank reports why.
#pragma once

#include <cstddef>
#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace dlnb {

// The message of the last Error constructed on this thread (read by the
// failure path of a GPU run while the exception is still unwinding, where
// std::current_exception() has nothing yet).
std::string& last_error_message();

class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& what) : std::runtime_error(what) { last_error_message() = what; }
};

#define DLNB_THROW(msg)                                                        \
  do {                                                                         \
    std::ostringstream dlnb_oss_;                                              \
    dlnb_oss_ << __FILE__ << ":" << __LINE__ << ": " << msg;                   \
    throw ::dlnb::Error(dlnb_oss_.str());                                      \
  } while (0)

#define DLNB_REQUIRE(cond, msg)                                                \
  do {                                                                         \
    if (!(cond)) DLNB_THROW("requirement failed: " #cond ": " << msg);         \
  } while (0)

// Element type of every buffer and of every collective on the wire.
enum class DType : int { BF16 = 0, FP16 = 1, FP32 = 2, FP8_E4M3 = 3, FP8_E5M2 = 4 };

size_t dtype_size(DType t);
const char* dtype_name(DType t);
DType parse_dtype(const std::string& s);  // accepts bf16/bfloat16/fp32/float/fp8/float8/...

// Where a strategy's buffers live and where its compute/collectives run.
enum class DeviceKind : int { CPU = 0, GPU = 1 };

// String helpers.
std::string trim(const std::string& s);
std::vector<std::string> split(const std::string& s, char sep);
bool starts_with(const std::string& s, const std::string& p);
bool ends_with(const std::string& s, const std::string& p);
std::string env_or(const char* name, const std::string& dflt);
long long env_int(const char* name, long long dflt);
// True in the CLI binaries (main_for), false when a host process (Python)
// runs the library: only a CLI process may end itself on a fatal error.
bool cli_process();

// Host-side bf16 / fp8 <-> float conversions (CPU backend reductions, tests).
float bf16_to_float(uint16_t v);
uint16_t float_to_bf16(float f);  // round-to-nearest-even, NaN preserving
float fp16_to_float(uint16_t v);
uint16_t float_to_fp16(float f);
float fp8e4m3_to_float(uint8_t v);  // OCP e4m3fn (gfx950 native), not fnuz
uint8_t float_to_fp8e4m3(float f);  // saturating
float fp8e5m2_to_float(uint8_t v);
uint8_t float_to_fp8e5m2(float f);

}  // namespace dlnb
