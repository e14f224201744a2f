// file_io.cpp — whole-file load/save and the FL / RL container formats.
//
// The FL container is byte-identical to the reference's (src/file_io.cu:222-280
// writes inputSize, bitsSize, valuesSize as host-endian u64 and then the two
// arrays; :117-192 reads them back). Loading additionally checks the declared
// sizes against the file length before allocating, so a truncated or corrupt
// header fails with a message instead of reading out of bounds. Saving writes a
// temporary file next to the output and renames it into place when complete
// (flrl_outfile.hpp), so a failed run never truncates or removes an existing
// output.
#include "file_io.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "flrl_outfile.hpp"

namespace flrl_cli {

namespace {

struct File {
    FILE *f = nullptr;
    explicit File(const char *path, const char *mode) : f(std::fopen(path, mode))
    {
        if (!f)
            throw std::runtime_error(std::string("[FileIO] Cannot open file: ") + path);
    }
    File() = default;
    ~File()
    {
        if (f)
            std::fclose(f);
    }
    size_t length()
    {
        if (std::fseek(f, 0, SEEK_END) != 0)
            throw std::runtime_error("[FileIO] Cannot seek file");
        const long end = std::ftell(f);
        if (end < 0 || std::fseek(f, 0, SEEK_SET) != 0)
            throw std::runtime_error("[FileIO] Cannot seek file");
        return (size_t)end;
    }
    void read(void *dst, size_t bytes)
    {
        if (bytes && std::fread(dst, 1, bytes, f) != bytes)
            throw std::runtime_error("[FileIO] Cannot read file content");
    }
    void write(const void *src, size_t bytes)
    {
        if (bytes && std::fwrite(src, 1, bytes, f) != bytes)
            throw std::runtime_error("[FileIO] Cannot write to file");
    }
    void close()
    {
        FILE *g = f;
        f = nullptr;
        if (std::fclose(g) != 0)
            throw std::runtime_error("[FileIO] Cannot write to file");
    }
};

// An output file: buffered writes into a temporary next to `path`, moved into
// place by close().
struct OutputFile {
    flrl::OutFile out;
    File file;
    explicit OutputFile(const char *path)
    {
        if (!out.open(path))
            throw std::runtime_error(std::string("[FileIO] Cannot open file: ") + path);
        file.f = fdopen(out.fd, "wb");
        if (!file.f)
            throw std::runtime_error(std::string("[FileIO] Cannot open file: ") + path);
        out.fd = -1;  // owned by the FILE from here on
    }
    void write(const void *src, size_t bytes) { file.write(src, bytes); }
    void close()
    {
        file.close();  // fclose: the descriptor is closed with the FILE
        if (!out.commit())
            throw std::runtime_error("[FileIO] Cannot write to file");
    }
};

uint8_t *alloc_bytes(size_t n)
{
    uint8_t *p = static_cast<uint8_t *>(std::malloc(n ? n : 1));
    if (!p)
        throw std::runtime_error("Cannot allocate memory");
    return p;
}

}  // namespace

FileData loadFile(const char *path)
{
    File f(path, "rb");
    FileData fd;
    fd.size = f.length();
    fd.data = alloc_bytes(fd.size);
    try {
        f.read(fd.data, fd.size);
    } catch (...) {
        std::free(fd.data);
        throw;
    }
    return fd;
}

void saveFile(const char *path, const FileData &fd)
{
    OutputFile f(path);
    f.write(fd.data, fd.size);
    f.close();
}

flrl_fl_buf loadCompressedFL(const char *path)
{
    File f(path, "rb");
    const size_t len = f.length();
    uint64_t hdr[3];
    if (len < sizeof(hdr))
        throw std::runtime_error("[FileIO] Cannot read file content (FL header truncated)");
    f.read(hdr, sizeof(hdr));
    flrl_fl_buf c{};
    c.input_size = hdr[0];
    c.bits_size = hdr[1];
    c.values_size = hdr[2];
    if (c.bits_size > len - sizeof(hdr) || c.values_size > len - sizeof(hdr) - c.bits_size)
        throw std::runtime_error("[FileIO] Cannot read file content (FL sizes exceed file)");
    c.bits = alloc_bytes(c.bits_size);
    c.values = static_cast<uint8_t *>(std::malloc(c.values_size ? c.values_size : 1));
    if (!c.values) {
        std::free(c.bits);
        throw std::runtime_error("Cannot allocate memory");
    }
    try {
        f.read(c.bits, c.bits_size);
        f.read(c.values, c.values_size);
    } catch (...) {
        std::free(c.bits);
        std::free(c.values);
        throw;
    }
    return c;
}

void saveCompressedFL(const char *path, const flrl_fl_buf &c)
{
    OutputFile f(path);
    const uint64_t hdr[3] = {c.input_size, c.bits_size, c.values_size};
    f.write(hdr, sizeof(hdr));
    f.write(c.bits, c.bits_size);
    f.write(c.values, c.values_size);
    f.close();
}

flrl_rl_buf loadCompressedRL(const char *path)
{
    File f(path, "rb");
    const size_t len = f.length();
    uint64_t hdr[2];
    if (len < sizeof(hdr))
        throw std::runtime_error("[FileIO] Cannot read file content (RL header truncated)");
    f.read(hdr, sizeof(hdr));
    flrl_rl_buf c{};
    c.input_size = hdr[0];
    c.runs = hdr[1];
    if (c.runs > (len - sizeof(hdr)) / 2 || len - sizeof(hdr) != 2 * c.runs)
        throw std::runtime_error("[FileIO] Cannot read file content (RL runs do not match file)");
    c.counts = alloc_bytes(c.runs);
    c.values = static_cast<uint8_t *>(std::malloc(c.runs ? c.runs : 1));
    if (!c.values) {
        std::free(c.counts);
        throw std::runtime_error("Cannot allocate memory");
    }
    try {
        f.read(c.counts, c.runs);
        f.read(c.values, c.runs);
    } catch (...) {
        std::free(c.counts);
        std::free(c.values);
        throw;
    }
    return c;
}

void saveCompressedRL(const char *path, const flrl_rl_buf &c)
{
    OutputFile f(path);
    const uint64_t hdr[2] = {c.input_size, c.runs};
    f.write(hdr, sizeof(hdr));
    f.write(c.counts, c.runs);
    f.write(c.values, c.runs);
    f.close();
}

}  // namespace flrl_cli
