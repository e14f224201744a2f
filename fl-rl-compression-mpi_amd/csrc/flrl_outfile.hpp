// flrl_outfile.hpp — output files that appear whole or not at all.
//
// The reference loads the whole input before it opens the output
// (src/main.cu:72-129, src/file_io.cu:194-280), so `compress c fl f f` works
// there and a failed run leaves an existing output alone. The streamed file
// paths here read the input while writing, so they write to a temporary file
// next to the output (same directory, so rename() is atomic on one file
// system) and rename it into place only on success; on failure the temporary
// is unlinked and a pre-existing output is untouched. The replacement keeps
// an existing output's mode (and owner where permitted), and a symlinked
// output's target is replaced, not the link. An existing output that is not a
// regular file (/dev/null, a FIFO) is written directly, and so is one whose
// directory does not allow a temporary (unless it is the input being read).
// EXCEPTION to "untouched": that in-place case truncates the existing output
// at open (as the reference's fopen(path, "wb") does), so a later failure
// leaves it truncated or partial. Callers therefore acquire every other
// resource that can fail up front (e.g. the RL side file) before open().
// Header-only (POSIX), shared by libflrl.so and the CLI.
#pragma once

#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <vector>

namespace flrl {

// Creation mode of a new output: 0666 & ~umask, as fopen(path, "wb") would
// give (read from /proc/self/status rather than set-and-restore umask, which
// would race other threads creating files).
inline mode_t new_file_mode()
{
    mode_t mask = 022;
    if (FILE *f = fopen("/proc/self/status", "r")) {
        char line[128];
        while (fgets(line, sizeof(line), f))
            if (strncmp(line, "Umask:", 6) == 0) {
                mask = (mode_t)strtoul(line + 6, nullptr, 8);
                break;
            }
        fclose(f);
    }
    return 0666 & ~mask;
}

class OutFile {
public:
    int fd = -1;

    OutFile() = default;
    OutFile(const OutFile &) = delete;
    OutFile &operator=(const OutFile &) = delete;
    ~OutFile()
    {
        if (fd >= 0)
            ::close(fd);
        if (!done_ && !tmp_.empty())
            ::unlink(tmp_.c_str());
    }

    // false (errno set) when the output cannot be created. input_fd: a file the
    // caller is still reading (never truncated in place, see below), or -1.
    bool open(const char *path, bool read_write = false, int input_fd = -1)
    {
        path_ = path;
        // an existing symlink's target is replaced, not the link itself (as
        // fopen(path, "wb") writes through it)
        if (char *rp = ::realpath(path, nullptr)) {
            path_ = rp;
            ::free(rp);
        }
        struct stat st;
        const bool exists = ::stat(path_.c_str(), &st) == 0;
        if (exists && !S_ISREG(st.st_mode)) {
            direct_ = true;
            fd = ::open(path_.c_str(), read_write ? O_RDWR : O_WRONLY);
            return fd >= 0;
        }
        const size_t slash = path_.rfind('/');
        const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : path_.substr(0, slash));
        const std::string base = slash == std::string::npos ? path_ : path_.substr(slash + 1);
        std::string t = dir + "/." + base + ".flrl-XXXXXX";
        std::vector<char> buf(t.begin(), t.end());
        buf.push_back('\0');
        fd = ::mkstemp(buf.data());
        if (fd < 0) {
            // no temporary possible (directory not writable): truncate and write
            // the existing output in place, as the reference does — unless it is
            // the input still being read
            const int e = errno;
            struct stat ist;
            const bool is_input = input_fd >= 0 && ::fstat(input_fd, &ist) == 0 && ist.st_dev == st.st_dev &&
                                  ist.st_ino == st.st_ino;
            if (exists && (e == EACCES || e == EPERM || e == EROFS) && !is_input) {
                fd = ::open(path_.c_str(), (read_write ? O_RDWR : O_WRONLY) | O_TRUNC);
                if (fd >= 0) {
                    direct_ = in_place_ = true;
                    return true;
                }
            }
            errno = e;
            return false;
        }
        tmp_ = buf.data();
        if (exists) {  // the replacement keeps the output's mode and, where allowed, owner
            (void)::fchmod(fd, st.st_mode & 07777);
            if (::fchown(fd, st.st_uid, st.st_gid) != 0)
                (void)::fchmod(fd, st.st_mode & 0777);  // no set-id bits under another owner
        } else {
            (void)::fchmod(fd, new_file_mode());
        }
        return true;
    }

    // set the file length (no-op for a non-regular output)
    bool truncate(uint64_t len) { return (direct_ && !in_place_) || ::ftruncate(fd, (off_t)len) == 0; }

    // close (unless the caller already did, fd = -1) and move into place;
    // false (nothing replaced) on failure
    bool commit()
    {
        if (fd >= 0) {
            const int f = fd;
            fd = -1;
            if (::close(f) != 0)
                return false;
        }
        if (!direct_ && ::rename(tmp_.c_str(), path_.c_str()) != 0)
            return false;
        done_ = true;
        return true;
    }

private:
    std::string path_, tmp_;
    bool direct_ = false, in_place_ = false, done_ = false;
};

// An anonymous scratch file in directory `dir` (unlinked at once, so it never
// collides with or clobbers a user file). -1 on failure.
inline int anon_file_in(const std::string &dir)
{
#ifdef O_TMPFILE
    const int t = ::open(dir.c_str(), O_TMPFILE | O_RDWR, 0600);
    if (t >= 0)
        return t;
#endif
    std::string s = dir + "/.flrl-side-XXXXXX";
    std::vector<char> buf(s.begin(), s.end());
    buf.push_back('\0');
    const int fd = ::mkstemp(buf.data());
    if (fd >= 0)
        ::unlink(buf.data());
    return fd;
}

// An anonymous scratch file next to `near_path` (same file system as the
// output), else in $TMPDIR or /tmp when that directory allows none (the
// read-only-directory case in which OutFile writes in place). -1 on failure.
inline int anon_file_near(const char *near_path)
{
    std::string p(near_path);
    const size_t slash = p.rfind('/');
    const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : p.substr(0, slash));
    int fd = anon_file_in(dir);
    if (fd >= 0)
        return fd;
    const char *td = ::getenv("TMPDIR");
    if (td && *td && (fd = anon_file_in(td)) >= 0)
        return fd;
    return anon_file_in("/tmp");
}

}  // namespace flrl
