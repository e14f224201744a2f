// cpu_codec.hpp — host-CPU codec behind the CLI's fl-cpu / rl-cpu methods
// (the reference's cpuCompress / cpuDecompress, src/fl/fl_cpu.cuh:9-10).
// Independent of oracle/ (which is test infrastructure only). Throws
// std::runtime_error on malformed input; returns malloc'd buffers.
#pragma once

#include <cstddef>
#include <cstdint>

#include "flrl.h"

namespace flrl_cli {

flrl_fl_buf cpuCompressFL(const uint8_t *data, size_t size, unsigned threads);
// Empty result (data == nullptr, size 0) on the reference's early-out
// valuesSize == 0 || bitsSize == 0 (fl_cpu.cu:94-97).
void cpuDecompressFL(const flrl_fl_buf &c, uint8_t **out, size_t *out_size, unsigned threads);

flrl_rl_buf cpuCompressRL(const uint8_t *data, size_t size);
void cpuDecompressRL(const flrl_rl_buf &c, uint8_t **out, size_t *out_size);

}  // namespace flrl_cli
