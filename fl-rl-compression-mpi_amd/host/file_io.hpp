// file_io.hpp — on-disk formats (reference: src/file_io.cuh, src/file_io.cu).
#pragma once

#include <cstddef>
#include <cstdint>

#include "flrl.h"

namespace flrl_cli {

// Owns a malloc'd byte buffer (released with free(), the reference's rule).
struct FileData {
    uint8_t *data = nullptr;
    size_t size = 0;
};

// All functions throw std::runtime_error with a "[FileIO] ..." message.
FileData loadFile(const char *path);                     // file_io.cu:73-115
void saveFile(const char *path, const FileData &fd);     // file_io.cu:194-220

// FL: u64 inputSize | u64 bitsSize | u64 valuesSize | bits | values
// (file_io.cu:222-280 write, :117-192 read; little-endian host order).
flrl_fl_buf loadCompressedFL(const char *path);
void saveCompressedFL(const char *path, const flrl_fl_buf &c);

// RL (build-defined): u64 inputSize | u64 runs | counts[runs] | values[runs]
flrl_rl_buf loadCompressedRL(const char *path);
void saveCompressedRL(const char *path, const flrl_rl_buf &c);

}  // namespace flrl_cli
