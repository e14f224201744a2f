// args_parser.cpp — command line of the `compress` CLI. Accepts the reference's
// methods (src/args_parser.cu:30-53: fl, fl-cpu, fl-mpi, fl-nccl, fl-shmem) plus
// the README's rl / rl-cpu (README.md:25-26), which the reference parser lacks.
// fl-mpi / fl-nccl / fl-shmem all select the single-process multi-GPU path
// (the reference's fl-shmem silently ran the CPU codec, main.cu:90-91,116-117).
#include "args_parser.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace flrl_cli {

Args parseArguments(int argc, char **argv)
{
    const char *prog = argc > 0 ? argv[0] : "compress";
    if (argc != 5)
        usage(prog);

    Operation op;
    if (std::strcmp(argv[1], "c") == 0)
        op = Operation::Compression;
    else if (std::strcmp(argv[1], "d") == 0)
        op = Operation::Decompression;
    else
        usage(prog);

    struct Entry {
        const char *name;
        Method method;
    };
    static const Entry kMethods[] = {
        {"fl", Method::FixedLength},          {"fl-cpu", Method::FixedLengthCPU},
        {"fl-mpi", Method::FixedLengthMulti}, {"fl-nccl", Method::FixedLengthMulti},
        {"fl-shmem", Method::FixedLengthMulti}, {"rl", Method::RunLength},
        {"rl-cpu", Method::RunLengthCPU},
    };
    for (const Entry &e : kMethods)
        if (std::strcmp(argv[2], e.name) == 0)
            return Args{op, e.method, e.name, argv[3], argv[4]};
    usage(prog);
}

void usage(const char *prog)
{
    std::fprintf(stderr, "USAGE: %s operation method input_file output_file\n", prog);
    std::fprintf(stderr, "operation - c (compress) or d (decompress)\n");
    std::fprintf(stderr,
                 "method - fl (fixed-length, one GPU), fl-cpu (fixed-length, CPU), "
                 "fl-mpi | fl-nccl | fl-shmem (fixed-length, all GPUs of the node), "
                 "rl (run-length, one GPU), rl-cpu (run-length, CPU)\n");
    std::exit(1);
}

}  // namespace flrl_cli
