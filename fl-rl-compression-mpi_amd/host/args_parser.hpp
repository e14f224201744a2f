// args_parser.hpp — `compress {c|d} <method> <in> <out>` (reference:
// src/args_parser.cuh:12-19, src/args_parser.cu:8-68).
#pragma once

namespace flrl_cli {

enum class Operation { Compression, Decompression };

enum class Method {
    FixedLength,       // fl        — one GPU (HIP)
    FixedLengthCPU,    // fl-cpu    — host CPU
    FixedLengthMulti,  // fl-mpi | fl-nccl | fl-shmem — all GPUs of the node (RCCL size-scan)
    RunLength,         // rl        — one GPU (HIP)
    RunLengthCPU,      // rl-cpu    — host CPU
};

struct Args {
    Operation operation;
    Method method;
    const char *methodName;
    const char *inputFile;
    const char *outputFile;
};

// Exits with status 1 after printing usage on any malformed command line
// (args_parser.cu:10-59,62-68).
Args parseArguments(int argc, char **argv);
[[noreturn]] void usage(const char *prog);

}  // namespace flrl_cli
