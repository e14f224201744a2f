// main.cpp — the `compress` CLI (reference: src/main.cu:18-169).
//
//   compress c <method> <input> <output>     compress a file
//   compress d <method> <input> <output>     decompress a file
//
// fl / fl-mpi / fl-nccl / fl-shmem / rl run on the GPU through the C ABI in
// include/flrl.h (libflrl.so); fl-cpu / rl-cpu run the host codec. The GPU
// methods stream the file through the GPUs in chunks (flrl_{fl,rl}_*_file:
// `fl` and `rl` one pipeline, the multi-GPU FL methods one per GPU), so
// neither the file nor its output is held in memory; FLRL_CHUNK_BYTES and FLRL_WORKERS override the chunk size (64 MiB)
// and the pipeline count. Errors print
// "[ERROR]: <message>" to stderr like the reference (main.cu:95-98), but the
// process then exits with status 2 instead of 0; no partial output file is
// left behind and an existing output is never truncated or removed (outputs
// are renamed into place when complete, so the input may also be the output). Phase timings print as the reference's "[TIMER]" lines.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>

#include "args_parser.hpp"
#include "cpu_codec.hpp"
#include "file_io.hpp"
#include "flrl.h"

using namespace flrl_cli;

namespace {

struct Timer {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void done(const char *step)
    {
        const double ms = std::chrono::duration<double, std::milli>(
                              std::chrono::steady_clock::now() - t0)
                              .count();
        std::printf("[TIMER] Step: \"%s\", Time: %.3f ms\n", step, ms);
        t0 = std::chrono::steady_clock::now();
    }
};

void check(int rc, const char *what)
{
    if (rc != FLRL_OK)
        throw std::runtime_error(std::string(what) + ": " + flrl_last_error());
}

unsigned host_threads()
{
    const unsigned h = std::thread::hardware_concurrency();
    return h ? h : 1;
}

size_t env_size(const char *name, size_t dflt)
{
    const char *v = std::getenv(name);
    return (v && *v) ? (size_t)std::strtoull(v, nullptr, 0) : dflt;
}

// FL / RL on the GPU(s), file to file: one call does load + encode/decode + save.
bool fl_streamed(const Args &a, bool compress_op)
{
    const bool rl = a.method == Method::RunLength;
    if (a.method != Method::FixedLength && a.method != Method::FixedLengthMulti && !rl)
        return false;
    const int workers = (int)env_size("FLRL_WORKERS", a.method == Method::FixedLengthMulti ? 0 : 1);
    const size_t chunk = env_size("FLRL_CHUNK_BYTES", 0);
    Timer t;
    if (rl && compress_op)
        check(flrl_rl_compress_file(a.inputFile, a.outputFile, workers, chunk), "rl compress");
    else if (rl)
        check(flrl_rl_decompress_file(a.inputFile, a.outputFile, workers, chunk), "rl decompress");
    else if (compress_op)
        check(flrl_fl_compress_file(a.inputFile, a.outputFile, workers, chunk), "fl compress");
    else
        check(flrl_fl_decompress_file(a.inputFile, a.outputFile, workers, chunk), "fl decompress");
    t.done(compress_op ? "Compression (streamed: load + encode + save)"
                       : "Decompression (streamed: load + decode + save)");
    return true;
}

// fl-cpu / rl-cpu: whole file in host memory, like the reference (main.cu:72-129).
void compress(const Args &a)
{
    if (fl_streamed(a, true))
        return;
    Timer t;
    FileData in = loadFile(a.inputFile);
    t.done("Load data from file");
    try {
        if (a.method == Method::FixedLengthCPU) {
            flrl_fl_buf c = cpuCompressFL(in.data, in.size, host_threads());
            t.done("Compression");
            try {
                saveCompressedFL(a.outputFile, c);
            } catch (...) {
                std::free(c.bits);
                std::free(c.values);
                throw;
            }
            std::free(c.bits);
            std::free(c.values);
        } else {
            flrl_rl_buf c = cpuCompressRL(in.data, in.size);
            t.done("Compression");
            try {
                saveCompressedRL(a.outputFile, c);
            } catch (...) {
                std::free(c.counts);
                std::free(c.values);
                throw;
            }
            std::free(c.counts);
            std::free(c.values);
        }
        t.done("Save data to file");
    } catch (...) {
        std::free(in.data);
        throw;
    }
    std::free(in.data);
}

// fl-cpu / rl-cpu (main.cu:131-169).
void decompress(const Args &a)
{
    if (fl_streamed(a, false))
        return;
    Timer t;
    FileData out;
    if (a.method == Method::FixedLengthCPU) {
        flrl_fl_buf c = loadCompressedFL(a.inputFile);
        t.done("Load data from file");
        try {
            cpuDecompressFL(c, &out.data, &out.size, host_threads());
        } catch (...) {
            std::free(c.bits);
            std::free(c.values);
            throw;
        }
        std::free(c.bits);
        std::free(c.values);
    } else {
        flrl_rl_buf c = loadCompressedRL(a.inputFile);
        t.done("Load data from file");
        try {
            cpuDecompressRL(c, &out.data, &out.size);
        } catch (...) {
            std::free(c.counts);
            std::free(c.values);
            throw;
        }
        std::free(c.counts);
        std::free(c.values);
    }
    t.done("Decompression");
    try {
        saveFile(a.outputFile, out);
    } catch (...) {
        std::free(out.data);
        throw;
    }
    std::free(out.data);
    t.done("Save data to file");
}

}  // namespace

int main(int argc, char **argv)
{
    const Args a = parseArguments(argc, argv);
    try {
        if (a.operation == Operation::Compression)
            compress(a);
        else
            decompress(a);
    } catch (const std::exception &e) {
        // outputs are written to a temporary and renamed into place only on
        // success (flrl_outfile.hpp), so there is nothing to clean up here: an
        // existing output file is left as it was
        std::fprintf(stderr, "[ERROR]: %s\n", e.what());
        return 2;
    }
    return 0;
}
