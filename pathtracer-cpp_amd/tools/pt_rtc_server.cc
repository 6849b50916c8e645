// pt_rtc_server — the scene kernel's hipRTC compiles, run in a child process of libpt_hip.so.
//
// Why a process ("Process exit during a background compile"): a compile on a
// background thread of the render process runs inside amd_comgr, whose lazily constructed
// statics register their destructors with atexit DURING the compile, i.e. after any handler
// the library could register to wait for it. A process that exits with a compile in flight
// therefore destroys them under the running compile (SIGSEGV at exit, reproduced on the CPU:
// tests/test_rtc_exit.py). Here the compile has a process of its own; the render process only
// writes a request to a socket and reads the code object back.
//
// usage: pt_rtc_server [--lib PATH]...   (libraries dlopen'ed first, in order: the caller passes
//        the amd_comgr and hiprtc libraries its own process would compile with)
// Protocol on fd 0 / fd 1 (one socket), repeated until end of input:
//   request : "PTRQ" u32 n_headers u32 n_options, then as (u64 length, bytes) strings: the
//             source, n_headers x (name, text), n_options x option
//   response: "PTRS" u32 ok, u64 length, bytes (the code object, or the compile log)
#include <dlfcn.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

namespace {

typedef int (*CreateFn)(void**, const char*, const char*, int, const char* const*, const char* const*);
typedef int (*CompileFn)(void*, int, const char* const*);
typedef int (*SizeFn)(void*, size_t*);
typedef int (*GetFn)(void*, char*);
typedef int (*DestroyFn)(void**);

struct Rtc {
    CreateFn create;
    CompileFn compile;
    SizeFn log_size, code_size;
    GetFn log, code;
    DestroyFn destroy;
};

bool read_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n > 0) {
        const ssize_t r = read(fd, c, n);
        if (r <= 0) return false;
        c += r;
        n -= (size_t)r;
    }
    return true;
}

bool write_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n > 0) {
        const ssize_t r = write(fd, c, n);
        if (r <= 0) return false;
        c += r;
        n -= (size_t)r;
    }
    return true;
}

bool read_str(int fd, std::string& s) {
    uint64_t n = 0;
    if (!read_all(fd, &n, 8) || n > ((uint64_t)1 << 30)) return false;
    s.resize(n);
    return n == 0 || read_all(fd, &s[0], n);
}

bool respond(bool ok, const std::vector<char>& bytes) {
    const uint32_t head[2] = {0x53525450u /* "PTRS" */, ok ? 1u : 0u};
    const uint64_t n = bytes.size();
    return write_all(1, head, 8) && write_all(1, &n, 8) && (n == 0 || write_all(1, bytes.data(), n));
}

template <typename F>
bool sym(void* h, const char* name, F& f) {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != nullptr;
}

}  // namespace

int main(int argc, char** argv) {
    signal(SIGPIPE, SIG_IGN);  // the render process went away: the write fails, we exit
    void* rtc = nullptr;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (strcmp(argv[i], "--lib") != 0) continue;
        void* h = dlopen(argv[i + 1], RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            fprintf(stderr, "pt_rtc_server: %s\n", dlerror());
            return 2;
        }
        if (dlsym(h, "hiprtcCompileProgram")) rtc = h;
    }
    if (!rtc) rtc = dlopen("libhiprtc.so", RTLD_NOW | RTLD_GLOBAL);
    Rtc f;
    if (!rtc || !sym(rtc, "hiprtcCreateProgram", f.create) || !sym(rtc, "hiprtcCompileProgram", f.compile) ||
        !sym(rtc, "hiprtcGetProgramLogSize", f.log_size) || !sym(rtc, "hiprtcGetProgramLog", f.log) ||
        !sym(rtc, "hiprtcGetCodeSize", f.code_size) || !sym(rtc, "hiprtcGetCode", f.code) ||
        !sym(rtc, "hiprtcDestroyProgram", f.destroy)) {
        fprintf(stderr, "pt_rtc_server: no hipRTC library\n");
        return 2;
    }
    while (true) {
        uint32_t head[3];
        if (!read_all(0, head, 12)) return 0;  // end of input: the render process is done
        if (head[0] != 0x51525450u /* "PTRQ" */ || head[1] > 16 || head[2] > 256) return 3;
        std::string src;
        std::vector<std::string> names(head[1]), hdrs(head[1]), opts(head[2]);
        bool ok = read_str(0, src);
        for (uint32_t i = 0; ok && i < head[1]; i++) ok = read_str(0, names[i]) && read_str(0, hdrs[i]);
        for (uint32_t i = 0; ok && i < head[2]; i++) ok = read_str(0, opts[i]);
        if (!ok) return 3;
        std::vector<const char*> np, hp, op;
        for (uint32_t i = 0; i < head[1]; i++) np.push_back(names[i].c_str()), hp.push_back(hdrs[i].c_str());
        for (const std::string& o : opts) op.push_back(o.c_str());
        void* prog = nullptr;
        std::vector<char> out;
        bool good = false;
        if (f.create(&prog, src.c_str(), "pt_trace_flat_rtc.hip", (int)head[1], hp.data(), np.data()) != 0) {
            const char msg[] = "hiprtcCreateProgram failed";
            out.assign(msg, msg + sizeof(msg) - 1);
        } else {
            if (f.compile(prog, (int)op.size(), op.data()) != 0) {
                size_t n = 0;
                f.log_size(prog, &n);
                out.resize(n);
                if (n) f.log(prog, out.data());
            } else {
                size_t n = 0;
                f.code_size(prog, &n);
                out.resize(n);
                good = n > 0 && f.code(prog, out.data()) == 0;
            }
            f.destroy(&prog);
        }
        if (!respond(good, out)) return 0;
    }
}
