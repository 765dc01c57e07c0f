// api.cpp — the C-ABI of libpj (include/pj.h). Host code only: argument
// checks, ownership, error translation; all graph work happens in the HIP
// kernels of parse.hip / graph.hip / sort.hip / bfs.hip / delta.hip.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <chrono>
#include <cstdio>
#include <thread>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "engine.h"
#include "internal.h"

namespace pj {

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

}  // namespace pj

struct pj_ctx {
    pj::Ctx c;
};
struct pj_graph {
    pj::Graph g;
};

using namespace pj;

namespace {

template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const pj::Error& e) {
        set_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error("host allocation failed");
        return PJ_ERR_OOM;
    } catch (const std::exception& e) {
        set_error(e.what());
        return PJ_ERR_HIP;
    } catch (...) {
        set_error("unknown error");
        return PJ_ERR_HIP;
    }
}

int arg_error(const char* msg) {
    set_error(msg);
    return PJ_ERR_ARG;
}

void bind(const Ctx& c) { PJ_HIP(hipSetDevice(c.device)); }

uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

i64 out_degree(const Graph& g, i64 v) {
    if (g.off64) {
        u64 h[2];
        PJ_HIP(hipMemcpy(h, g.row64.p + v, sizeof(h), hipMemcpyDeviceToHost));
        return (i64)(h[1] - h[0]);
    }
    u32 h[2];
    PJ_HIP(hipMemcpy(h, g.row32.p + v, sizeof(h), hipMemcpyDeviceToHost));
    return (i64)(h[1] - h[0]);
}

// The file straight into HBM: reader threads pread fixed pieces into pinned
// staging slots (two per thread, kept in the ctx) and queue each piece's H2D copy
// as soon as it is read, so the disk / page-cache read and the PCIe copy overlap
// and no whole-file host buffer is allocated, faulted in and freed (the reference
// reads the file line by line, :66-105). The device buffer is zero-padded to
// padded_text_bytes(len) for the parser. A missing or unopenable file or a
// directory reads as empty (the reference does not check its ifstream, :67); a
// file that shrinks while being read is PJ_ERR_IO. Returns len.
constexpr int64_t kStageSlot = (int64_t)8 << 20;

void ensure_stage(Ctx& c, int slots) {
    while ((int)c.stage.size() < slots) {
        char* p = nullptr;
        hipEvent_t e = nullptr;
        PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&p), (size_t)kStageSlot, hipHostMallocDefault));
        PJ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c.stage.push_back(p);
        c.stage_ev.push_back(e);
    }
}

// Device -> pageable host copy through the ctx's pinned slots: up to 8 host threads,
// each copying its pieces into its own two slots (piece k + 1 in flight while piece k
// is moved out), so the PCIe copy and the host memcpy overlap. A plain hipMemcpy into
// pageable memory took 38 ms for the first 16.8 MB (K22 distances) of a process.
// host memory the HIP runtime knows as pinned (pj_host_pin, hipHostMalloc)
static bool host_pinned(const void* p) {
    hipPointerAttribute_t at{};
    const bool pinned = hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost;
    (void)hipGetLastError();  // (pageable memory reports an error here)
    return pinned;
}

void copy_d2h_staged(Ctx& c, void* host, const void* dev, size_t bytes) {
    if (bytes >= ((size_t)1 << 20) && host_pinned(host) && host_pinned(static_cast<char*>(host) + bytes - 1)) {
        PJ_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, c.stream));  // one DMA
        PJ_HIP(hipStreamSynchronize(c.stream));
        return;
    }
    if (bytes < ((size_t)1 << 20)) {
        if (bytes) PJ_HIP(hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost));
        return;
    }
    const size_t piece = (size_t)kStageSlot, np = (bytes + piece - 1) / piece;
    const int nt = (int)std::max<size_t>(1, std::min<size_t>(np, std::min(8u, std::thread::hardware_concurrency())));
    ensure_stage(c, 2 * nt);
    hipStream_t s = c.stream;
    std::vector<std::exception_ptr> errs((size_t)nt);
    auto work = [&](int t) {
        try {
            bind(c);
            auto issue = [&](size_t k, int slot) {
                const size_t off = k * piece, len = std::min(piece, bytes - off);
                PJ_HIP(hipMemcpyAsync(c.stage[(size_t)slot], static_cast<const char*>(dev) + off, len,
                                      hipMemcpyDeviceToHost, s));
                PJ_HIP(hipEventRecord(c.stage_ev[(size_t)slot], s));
            };
            int j = 0;
            if ((size_t)t < np) issue((size_t)t, 2 * t);
            for (size_t k = (size_t)t; k < np; k += (size_t)nt, ++j) {
                if (k + (size_t)nt < np) issue(k + (size_t)nt, 2 * t + ((j + 1) & 1));
                const int slot = 2 * t + (j & 1);
                PJ_HIP(hipEventSynchronize(c.stage_ev[(size_t)slot]));
                const size_t off = k * piece, len = std::min(piece, bytes - off);
                std::memcpy(static_cast<char*>(host) + off, c.stage[(size_t)slot], len);
            }
        } catch (...) {
            errs[(size_t)t] = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
}

i64 read_file_to_device(Ctx& c, const char* path, DevBuf<uint8_t>& text) {
    hipStream_t s = c.stream;
    struct stat sb;
    int fd = -1;
    int64_t size = 0;
    if (stat(path, &sb) == 0 && S_ISREG(sb.st_mode) && sb.st_size > 0 && (fd = open(path, O_RDONLY)) >= 0)
        size = (int64_t)sb.st_size;
    const i64 padded = padded_text_bytes(size);
    text.alloc((size_t)padded);
    PJ_HIP(hipMemsetAsync(text.p + size, 0, (size_t)(padded - size), s));
    if (size == 0) {
        if (fd >= 0) close(fd);
        PJ_HIP(hipStreamSynchronize(s));
        return 0;
    }
    const int64_t npieces = (size + kStageSlot - 1) / kStageSlot;
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(npieces, std::min(8u, std::thread::hardware_concurrency())));
    ensure_stage(c, 2 * nt);
    std::atomic<int64_t> got{0};
    std::vector<std::exception_ptr> errs((size_t)nt);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            try {
                bind(c);
                const bool warm = t == nt - 1 && npieces > 1;
                if (warm) {
                    // warm the device -> host copy path while the others read: the first D2H
                    // of a process pays a one-time ~10 ms setup (the distances come back
                    // this way after the solve)
                    PJ_HIP(hipMemcpyAsync(c.stage[(size_t)(2 * t + 1)], text.p + size - 1, 1, hipMemcpyDeviceToHost, s));
                    PJ_HIP(hipMemcpyAsync(c.stage[(size_t)(2 * t + 1)], text.p, std::min<int64_t>(size, (int64_t)2 << 20),
                                          hipMemcpyDeviceToHost, s));
                    PJ_HIP(hipEventRecord(c.stage_ev[(size_t)(2 * t + 1)], s));  // slot 2t+1 is busy until then
                }
                int k = 0;
                for (int64_t piece = t; piece < npieces; piece += nt, ++k) {
                    const int slot = 2 * t + (k & 1);
                    if (k >= 2 || (k == 1 && warm)) PJ_HIP(hipEventSynchronize(c.stage_ev[(size_t)slot]));  // its last copy is done
                    const int64_t off = piece * kStageSlot, want = std::min(kStageSlot, size - off);
                    char* buf = c.stage[(size_t)slot];
                    int64_t done = 0;
                    while (done < want) {
                        const ssize_t r = pread(fd, buf + done, (size_t)(want - done), (off_t)(off + done));
                        if (r <= 0) break;
                        done += r;
                    }
                    got.fetch_add(done);
                    if (done < want) break;
                    PJ_HIP(hipMemcpyAsync(text.p + off, buf, (size_t)want, hipMemcpyHostToDevice, s));
                    PJ_HIP(hipEventRecord(c.stage_ev[(size_t)slot], s));
                }
            } catch (...) {
                errs[(size_t)t] = std::current_exception();
            }
        });
    for (auto& x : th) x.join();
    close(fd);
    PJ_HIP(hipStreamSynchronize(s));
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    if (got.load() != size) throw Error(PJ_ERR_IO, std::string("short read of ") + path);
    return size;
}

void parse_error(const ParseResult& r) {
    set_error("edge list line " + std::to_string(r.bad_line) +
              ": second field missing, negative id or id out of range "
              "(undefined behaviour in the reference's read_webgraph)");
}

int finish_graph(pj_ctx* ctx, std::unique_ptr<pj_graph>& pg, pj_graph** out) {
    (void)ctx;
    *out = pg.release();
    return PJ_OK;
}

size_t format_rows(const int32_t* d, int64_t a, int64_t b, char* o) {
    size_t k = 0;
    for (int64_t i = a; i < b; ++i) {
        int32_t x = d[i];
        if (x == PJ_INT_INF) {
            o[k++] = 'i';
            o[k++] = 'n';
            o[k++] = 'f';
        } else {
            char rev[12];
            int r = 0;
            long long y = x;
            const bool neg = y < 0;
            if (neg) y = -y;
            do {
                rev[r++] = (char)('0' + y % 10);
                y /= 10;
            } while (y);
            if (neg) o[k++] = '-';
            while (r) o[k++] = rev[--r];
        }
        o[k++] = '\n';
    }
    return k;
}


// D2H of batch rows into pinned groups (double-buffered) and a pool of host
// threads that format and write one sol_file per row (output_vector :32-46,
// the bytes of pj_write_sol), overlapped with the next rows' GPU work.
class BatchWriter {
  public:
    BatchWriter(size_t n, const char* const* paths, bool strict, std::atomic<int>* err)
        : n_(n), paths_in_(paths), strict_(strict), err_(err) {
        const size_t row_bytes = std::max<size_t>(4 * n, 4);
        group_ = (int)std::max<size_t>(1, std::min<size_t>(256, ((size_t)256 << 20) / row_bytes));
        for (auto& b : buf_) b.alloc(row_bytes / 4 * (size_t)group_);
        nthreads_ = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    }
    ~BatchWriter() { join(); }
    void add_row(int idx, const int32_t* dev_row, hipStream_t s = nullptr) {
        if (fill_ == 0) join_slot(cur_);
        if (n_) {
            PJ_HIP(hipMemcpyAsync(buf_[cur_].p + (size_t)fill_ * n_, dev_row, 4 * n_, hipMemcpyDeviceToHost, s));
            PJ_HIP(hipStreamSynchronize(s));
        }
        paths_[cur_].push_back(paths_in_[idx]);
        if (++fill_ == group_) flush();
    }
    void finish() {
        if (fill_) flush();
        join();
    }
    std::string error() {
        std::lock_guard<std::mutex> lk(mu_);
        return msg_;
    }

  private:
    void flush() {
        const int slot = cur_, k = fill_;
        for (int t = 0; t < nthreads_ && t < k; ++t)
            th_[slot].emplace_back([this, slot, k, t] {
                std::vector<char> out(n_ * 12 + 16);
                for (int r = t; r < k; r += nthreads_) write_one(buf_[slot].p + (size_t)r * n_, paths_[slot][r], out);
            });
        cur_ ^= 1;
        fill_ = 0;
    }
    void write_one(const int32_t* d, const std::string& path, std::vector<char>& out) {
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) {
            if (strict_) fail(PJ_ERR_IO, "cannot open " + path);
            return;
        }
        static const char hdr[] = "the vector is:\n";
        size_t k = sizeof(hdr) - 1;
        std::memcpy(out.data(), hdr, k);
        k += format_rows(d, 0, (int64_t)n_, out.data() + k);
        const bool ok = std::fwrite(out.data(), 1, k, f) == k;
        if ((std::fclose(f) != 0 || !ok) && strict_) fail(PJ_ERR_IO, "write failed: " + path);
    }
    void fail(int code, const std::string& m) {
        std::lock_guard<std::mutex> lk(mu_);
        if (err_->load() == PJ_OK) {
            err_->store(code);
            msg_ = m;
        }
    }
    void join_slot(int slot) {
        for (auto& t : th_[slot]) t.join();
        th_[slot].clear();
        paths_[slot].clear();
    }
    void join() {
        join_slot(0);
        join_slot(1);
    }
    size_t n_;
    const char* const* paths_in_;
    bool strict_;
    std::atomic<int>* err_;
    int group_ = 1, nthreads_ = 1, cur_ = 0, fill_ = 0;
    PinnedBuf<int32_t> buf_[2];
    std::vector<std::string> paths_[2];
    std::vector<std::thread> th_[2];
    std::mutex mu_;
    std::string msg_;
};

}  // namespace

extern "C" {

const char* pj_last_error(void) { return g_err.c_str(); }

const char* pj_version(void) { return "libpj 0.1 (gfx950)"; }

int pj_trim_device_cache(int64_t* released) {
    return guarded([&] {
        const size_t r = dev_trim();
        if (released) *released = (int64_t)r;
        return PJ_OK;
    });
}

int pj_device_count(int* out) {
    if (!out) return arg_error("pj_device_count: out is NULL");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    *out = count;
    return PJ_OK;
}

int pj_create(int device, pj_ctx** out) {
    if (!out) return arg_error("pj_create: out is NULL");
    *out = nullptr;
    return guarded([&] {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
            set_error("no HIP device visible");
            return (int)PJ_ERR_NODEVICE;
        }
        if (device < 0 || device >= count) {
            set_error("device ordinal out of range");
            return (int)PJ_ERR_NODEVICE;
        }
        hipDeviceProp_t prop;
        PJ_HIP(hipGetDeviceProperties(&prop, device));
        if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
            set_error(std::string("libpj is built for gfx950 only; device is ") + prop.gcnArchName);
            return (int)PJ_ERR_NODEVICE;
        }
        auto c = std::make_unique<pj_ctx>();
        c->c.device = device;
        c->c.cu_count = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
        PJ_HIP(hipSetDevice(device));
        PJ_HIP(hipStreamCreateWithFlags(&c->c.own_stream, hipStreamNonBlocking));
        c->c.stream = c->c.own_stream;
        *out = c.release();
        return (int)PJ_OK;
    });
}

int pj_destroy(pj_ctx* ctx) {
    if (!ctx) return PJ_OK;
    return guarded([&] {
        bind(ctx->c);
        for (char* p : ctx->c.stage) (void)hipHostFree(p);
        for (hipEvent_t e : ctx->c.stage_ev) (void)hipEventDestroy(e);
        if (ctx->c.own_stream) (void)hipStreamDestroy(ctx->c.own_stream);
        delete ctx;
        return (int)PJ_OK;
    });
}

void* pj_stream(pj_ctx* ctx) { return ctx ? (void*)ctx->c.stream : nullptr; }

int pj_set_stream(pj_ctx* ctx, void* stream) {
    if (!ctx) return arg_error("pj_set_stream: ctx is NULL");
    return guarded([&] {
        bind(ctx->c);
        PJ_HIP(hipStreamSynchronize(ctx->c.stream));  // finish work queued on the previous stream
        ctx->c.stream = stream ? (hipStream_t)stream : ctx->c.own_stream;
        return (int)PJ_OK;
    });
}

namespace {

// COO from the parser -> CSR (+ CSC) on the device; csr_ms includes the kernels' completion
int graph_from_parse(pj_ctx* ctx, const ParseResult& r, DevBuf<u32>& src, DevBuf<u32>& dst, DevBuf<u32>& w,
                     int weighted, int64_t len, pj_graph** out) {
    if (r.bad_line) {
        parse_error(r);
        return (int)PJ_ERR_PARSE;
    }
    auto pg = std::make_unique<pj_graph>();
    pg->g.ctx = &ctx->c;
    const auto t0 = std::chrono::steady_clock::now();
    build_graph_from_coo(pg->g, src, dst, weighted ? &w : nullptr, r.nnz, r.max_id + 1, false);
    PJ_HIP(hipStreamSynchronize(ctx->c.stream));
    pg->g.load.csr_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    pg->g.load.h2d_ms = r.h2d_ms;
    pg->g.load.parse_ms = r.parse_ms;
    pg->g.load.text_bytes = len;
    return finish_graph(ctx, pg, out);
}

}  // namespace

int pj_load_snap_buffer(pj_ctx* ctx, const char* text, int64_t len, int weighted, pj_graph** out) {
    if (!ctx || !out || (len > 0 && !text) || len < 0) return arg_error("pj_load_snap_buffer: bad argument");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        DevBuf<u32> src, dst, w;
        ParseResult r = parse_snap_device(ctx->c, text, len, weighted != 0, src, dst, w);
        return graph_from_parse(ctx, r, src, dst, w, weighted, len, out);
    });
}

int pj_graph_load_stats(const pj_graph* g, pj_load_stats* out) {
    if (!g || !out) return arg_error("pj_graph_load_stats: bad argument");
    *out = g->g.load;
    return PJ_OK;
}

int pj_load_snap(pj_ctx* ctx, const char* path, int weighted, pj_graph** out) {
    if (!ctx || !path || !out) return arg_error("pj_load_snap: bad argument");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        const auto t0 = std::chrono::steady_clock::now();
        // A missing or unreadable file (or a directory) reads as empty, like the
        // reference's unchecked ifstream (:67): N = 0, header-only sol_file.
        DevBuf<uint8_t> text;
        const i64 len = read_file_to_device(ctx->c, path, text);
        const double read_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        DevBuf<u32> src, dst, w;
        ParseResult r = parse_device_text(ctx->c, text.p, len, weighted != 0, src, dst, w);
        text.release();
        const int rc = graph_from_parse(ctx, r, src, dst, w, weighted, len, out);
        if (rc == PJ_OK) (*out)->g.load.read_ms = read_ms;  // file -> HBM (read and H2D overlapped)
        return rc;
    });
}

int pj_load_coo(pj_ctx* ctx, const int64_t* src, const int64_t* dst, const uint32_t* w, int64_t nnz,
                int64_t n_vertices, pj_graph** out) {
    if (!ctx || !out || nnz < 0 || (nnz > 0 && (!src || !dst))) return arg_error("pj_load_coo: bad argument");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        std::vector<u32> hs((size_t)nnz), hd((size_t)nnz);
        i64 mx = -1;
        for (i64 i = 0; i < nnz; ++i) {
            const i64 a = src[i], b = dst[i];
            if (a < 0 || b < 0 || a > 0xFFFFFFFEll || b > 0xFFFFFFFEll) {
                set_error("pj_load_coo: vertex id out of range at edge " + std::to_string(i));
                return (int)PJ_ERR_RANGE;
            }
            hs[(size_t)i] = (u32)a;
            hd[(size_t)i] = (u32)b;
            mx = std::max(mx, std::max(a, b));
        }
        i64 n = n_vertices < 0 ? mx + 1 : n_vertices;
        if (n <= mx || n > 0xFFFFFFFFll) {
            set_error("pj_load_coo: n_vertices must exceed every id and fit 32 bits");
            return (int)PJ_ERR_RANGE;
        }
        hipStream_t s = ctx->c.stream;
        DevBuf<u32> ds((size_t)nnz), dd((size_t)nnz), dw;
        if (nnz) {
            PJ_HIP(hipMemcpyAsync(ds.p, hs.data(), 4 * (size_t)nnz, hipMemcpyHostToDevice, s));
            PJ_HIP(hipMemcpyAsync(dd.p, hd.data(), 4 * (size_t)nnz, hipMemcpyHostToDevice, s));
        }
        if (w) {
            dw.alloc((size_t)nnz);
            if (nnz) PJ_HIP(hipMemcpyAsync(dw.p, w, 4 * (size_t)nnz, hipMemcpyHostToDevice, s));
        }
        PJ_HIP(hipStreamSynchronize(s));
        auto pg = std::make_unique<pj_graph>();
        pg->g.ctx = &ctx->c;
        build_graph_from_coo(pg->g, ds, dd, w ? &dw : nullptr, nnz, n, false);
        return finish_graph(ctx, pg, out);
    });
}

int pj_generate_kronecker(pj_ctx* ctx, int scale, int edgefactor, uint64_t seed, int weighted, pj_graph** out) {
    if (!ctx || !out || scale < 0 || scale > 31 || edgefactor < 1 || edgefactor > 1024)
        return arg_error("pj_generate_kronecker: scale must be in [0,31], edgefactor in [1,1024]");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        DevBuf<u32> src, dst, w;
        generate_kronecker_device(ctx->c, scale, edgefactor, seed, weighted != 0, src, dst, weighted ? &w : nullptr);
        const i64 nnz = 2 * ((i64)edgefactor << scale);
        auto pg = std::make_unique<pj_graph>();
        pg->g.ctx = &ctx->c;
        build_graph_from_coo(pg->g, src, dst, weighted ? &w : nullptr, nnz, (i64)1 << scale, true);
        return finish_graph(ctx, pg, out);
    });
}

int pj_generate_webgraph(pj_ctx* ctx, int64_t n_ids, int64_t n_edges, uint64_t seed, pj_graph** out) {
    if (!ctx || !out || n_ids < 2 || n_ids > 0xFFFFFFFEll || n_edges < 1)
        return arg_error("pj_generate_webgraph: n_ids must be in [2, 2^32-2], n_edges >= 1");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        DevBuf<u32> src, dst;
        generate_webgraph_device(ctx->c, n_ids, n_edges, seed, src, dst);
        auto pg = std::make_unique<pj_graph>();
        pg->g.ctx = &ctx->c;
        build_graph_from_coo(pg->g, src, dst, nullptr, n_edges, n_ids, false);
        return finish_graph(ctx, pg, out);
    });
}

int pj_kronecker_write_snap(pj_ctx* ctx, int scale, int edgefactor, uint64_t seed, int weighted, const char* path) {
    if (!ctx || !path || scale < 0 || scale > 31 || edgefactor < 1 || edgefactor > 1024)
        return arg_error("pj_kronecker_write_snap: bad argument");
    return guarded([&] {
        bind(ctx->c);
        DevBuf<u32> src, dst, w;
        generate_kronecker_device(ctx->c, scale, edgefactor, seed, weighted != 0, src, dst, weighted ? &w : nullptr);
        const i64 nnz = 2 * ((i64)edgefactor << scale);
        FILE* f = std::fopen(path, "wb");
        if (!f) {
            set_error(std::string("pj_kronecker_write_snap: cannot open ") + path);
            return (int)PJ_ERR_IO;
        }
        std::unique_ptr<FILE, int (*)(FILE*)> fc(f, std::fclose);
        const char hdr[] = "# Graph500 Kronecker (A,B,C = 0.57,0.19,0.19), both directions\n# FromNodeId\tToNodeId\n";
        std::fwrite(hdr, 1, sizeof(hdr) - 1, f);
        const i64 chunk = (i64)1 << 24;
        const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<u32> hs((size_t)chunk), hd((size_t)chunk), hw(weighted ? (size_t)chunk : 0);
        std::vector<std::vector<char>> out(nt);
        std::vector<size_t> lens(nt);
        for (i64 c0 = 0; c0 < nnz; c0 += chunk) {
            const i64 k = std::min(chunk, nnz - c0);
            PJ_HIP(hipMemcpy(hs.data(), src.p + c0, 4 * (size_t)k, hipMemcpyDeviceToHost));
            PJ_HIP(hipMemcpy(hd.data(), dst.p + c0, 4 * (size_t)k, hipMemcpyDeviceToHost));
            if (weighted) PJ_HIP(hipMemcpy(hw.data(), w.p + c0, 4 * (size_t)k, hipMemcpyDeviceToHost));
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nt; ++t)
                th.emplace_back([&, t] {
                    const i64 a = k * t / nt, b = k * (t + 1) / nt;
                    out[t].resize((size_t)(b - a) * 36);
                    char* o = out[t].data();
                    size_t q = 0;
                    auto put = [&](u32 x) {
                        char rev[12];
                        int r = 0;
                        do {
                            rev[r++] = (char)('0' + x % 10);
                            x /= 10;
                        } while (x);
                        while (r) o[q++] = rev[--r];
                    };
                    for (i64 i = a; i < b; ++i) {
                        put(hs[(size_t)i]);
                        o[q++] = '\t';
                        put(hd[(size_t)i]);
                        if (weighted) {
                            o[q++] = '\t';
                            put(hw[(size_t)i]);
                        }
                        o[q++] = '\n';
                    }
                    lens[t] = q;
                });
            for (auto& t : th) t.join();
            for (unsigned t = 0; t < nt; ++t)
                if (std::fwrite(out[t].data(), 1, lens[t], f) != lens[t])
                    throw Error(PJ_ERR_IO, "pj_kronecker_write_snap: write failed");
        }
        if (std::fclose(fc.release()) != 0) throw Error(PJ_ERR_IO, "pj_kronecker_write_snap: write failed");
        return (int)PJ_OK;
    });
}

int pj_graph_destroy(pj_graph* g) {
    if (!g) return PJ_OK;
    return guarded([&] {
        bind(*g->g.ctx);
        delete g;
        return (int)PJ_OK;
    });
}

int pj_graph_info(const pj_graph* g, int64_t* n, int64_t* nnz, int* weighted, int* symmetric) {
    if (!g) return arg_error("pj_graph_info: graph is NULL");
    if (n) *n = g->g.n;
    if (nnz) *nnz = g->g.nnz;
    if (weighted) *weighted = g->g.weighted ? 1 : 0;
    if (symmetric) *symmetric = g->g.symmetric ? 1 : 0;
    return PJ_OK;
}

int pj_graph_get_csr(const pj_graph* pg, int64_t* row_ptr, int32_t* col, uint32_t* w) {
    if (!pg) return arg_error("pj_graph_get_csr: graph is NULL");
    return guarded([&] {
        const Graph& g = pg->g;
        bind(*g.ctx);
        if (row_ptr) {
            if (g.off64) {
                PJ_HIP(hipMemcpy(row_ptr, g.row64.p, 8 * (size_t)(g.n + 1), hipMemcpyDeviceToHost));
            } else {
                std::vector<u32> tmp((size_t)g.n + 1);
                PJ_HIP(hipMemcpy(tmp.data(), g.row32.p, 4 * (size_t)(g.n + 1), hipMemcpyDeviceToHost));
                for (size_t i = 0; i < tmp.size(); ++i) row_ptr[i] = tmp[i];
            }
        }
        if (col && g.nnz) PJ_HIP(hipMemcpy(col, g.col.p, 4 * (size_t)g.nnz, hipMemcpyDeviceToHost));
        if (w && g.nnz) {
            if (g.weighted) PJ_HIP(hipMemcpy(w, g.w.p, 4 * (size_t)g.nnz, hipMemcpyDeviceToHost));
            else std::fill(w, w + g.nnz, 1u);
        }
        return (int)PJ_OK;
    });
}

int pj_graph_out_degree(const pj_graph* g, int64_t v, int64_t* deg) {
    if (!g || !deg) return arg_error("pj_graph_out_degree: bad argument");
    if (v < 0 || v >= g->g.n) return arg_error("pj_graph_out_degree: vertex out of range");
    return guarded([&] {
        bind(*g->g.ctx);
        *deg = out_degree(g->g, v);
        return (int)PJ_OK;
    });
}

int pj_sample_roots(const pj_graph* g, uint64_t seed, int n, int64_t* roots, int* found) {
    if (!g || !roots || !found || n < 0) return arg_error("pj_sample_roots: bad argument");
    return guarded([&] {
        bind(*g->g.ctx);
        int k = 0;
        const i64 N = g->g.n;
        for (uint64_t c = 0; k < n && N > 0 && c < (uint64_t)n * 4096ull; ++c) {
            const i64 v = (i64)(splitmix64(seed + c) % (uint64_t)N);
            if (out_degree(g->g, v) < 1) continue;
            if (std::find(roots, roots + k, v) != roots + k) continue;
            roots[k++] = v;
        }
        *found = k;
        return (int)PJ_OK;
    });
}

int pj_sssp(pj_graph* pg, int64_t source, int32_t* dist_out) {
    if (!pg) return arg_error("pj_sssp: graph is NULL");
    return guarded([&] {
        Graph& g = pg->g;
        bind(*g.ctx);
        auto t0 = std::chrono::steady_clock::now();
        g.batch_stats = false;
        if (g.weighted) delta_solve(g, source);
        else bfs_solve(g, source);
        g.last_source = source;
        if (dist_out && g.n) {
            delta_materialize(g);
            copy_d2h_staged(*g.ctx, dist_out, g.dist.p, 4 * (size_t)g.n);
        }
        g.stats.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return (int)PJ_OK;
    });
}

int pj_copy_dist(pj_graph* pg, int32_t* dist_out) {
    if (!pg || (!dist_out && pg->g.n > 0)) return arg_error("pj_copy_dist: bad argument");
    if (!pg->g.have_result) {
        set_error("pj_copy_dist: no solve has run on this graph");
        return PJ_ERR_STATE;
    }
    return guarded([&] {
        bind(*pg->g.ctx);
        delta_materialize(pg->g);
        if (pg->g.n) copy_d2h_staged(*pg->g.ctx, dist_out, pg->g.dist.p, 4 * (size_t)pg->g.n);
        return (int)PJ_OK;
    });
}

int pj_host_pin(void* p, size_t bytes) {
    if (!p || !bytes) return arg_error("pj_host_pin: bad argument");
    return guarded([&] {
        PJ_HIP(hipHostRegister(p, bytes, hipHostRegisterDefault));
        return (int)PJ_OK;
    });
}

int pj_host_unpin(void* p) {
    if (!p) return arg_error("pj_host_unpin: bad argument");
    return guarded([&] {
        PJ_HIP(hipHostUnregister(p));
        return (int)PJ_OK;
    });
}

const int32_t* pj_dist_device(pj_graph* pg) {
    if (!pg || !pg->g.have_result) return nullptr;
    const int rc = guarded([&] {
        bind(*pg->g.ctx);
        delta_materialize(pg->g);  // (complete when it returns)
        return (int)PJ_OK;
    });
    return rc == PJ_OK ? pg->g.dist.p : nullptr;
}

// ---- shortest-path tree (tree.hip) ---------------------------------------------

int pj_parent_tree(pj_graph* pg, int64_t* parent_out) {
    if (!pg || (!parent_out && pg->g.n > 0)) return arg_error("pj_parent_tree: bad argument");
    if (!pg->g.have_result) {
        set_error("pj_parent_tree: no single-source solve has run on this graph");
        return PJ_ERR_STATE;
    }
    return guarded([&] {
        bind(*pg->g.ctx);
        delta_materialize(pg->g);
        parent_tree(pg->g, pg->g.last_source, parent_out);
        return (int)PJ_OK;
    });
}

int pj_validate_tree(pj_graph* pg, int64_t source, const int64_t* parent, pj_tree_report* out) {
    if (!pg || !out || (!parent && pg->g.n > 0)) return arg_error("pj_validate_tree: bad argument");
    if (!pg->g.have_result || pg->g.last_source != source) {
        set_error("pj_validate_tree: the last solve on this graph is not a single-source solve from source");
        return PJ_ERR_STATE;
    }
    return guarded([&] {
        bind(*pg->g.ctx);
        delta_materialize(pg->g);
        validate_tree(pg->g, source, parent, out);
        return (int)PJ_OK;
    });
}

int pj_write_parents(const int64_t* parent, int64_t n, const char* path) {
    if (!path || n < 0 || (n > 0 && !parent)) return arg_error("pj_write_parents: bad argument");
    return guarded([&] {
        FILE* f = std::fopen(path, "wb");
        if (!f) {
            set_error(std::string("cannot open ") + path);
            return (int)PJ_ERR_IO;
        }
        static const char hdr[] = "the parent tree is:\n";
        std::fwrite(hdr, 1, sizeof(hdr) - 1, f);
        std::vector<char> buf((size_t)1 << 20);
        size_t k = 0;
        for (int64_t v = 0; v < n; ++v) {
            if (k + 24 > buf.size()) {
                std::fwrite(buf.data(), 1, k, f);
                k = 0;
            }
            k += (size_t)std::snprintf(buf.data() + k, 24, "%lld\n", (long long)parent[v]);
        }
        std::fwrite(buf.data(), 1, k, f);
        if (std::fclose(f) != 0) {
            set_error(std::string("write failed: ") + path);
            return (int)PJ_ERR_IO;
        }
        return (int)PJ_OK;
    });
}

int pj_sssp_batch(pj_graph* pg, const int64_t* sources, int n_src, int32_t* dist_out) {
    if (!pg || (n_src > 0 && !sources) || n_src < 0) return arg_error("pj_sssp_batch: bad argument");
    return guarded([&] {
        Graph& g = pg->g;
        bind(*g.ctx);
        if (g.weighted) {
            delta_batch(g, sources, n_src, g.batch_streams, [&](int i, const int32_t* dev, hipStream_t s) {
                if (dist_out && g.n) {
                    PJ_HIP(hipMemcpyAsync(dist_out + (size_t)i * (size_t)g.n, dev, 4 * (size_t)g.n,
                                          hipMemcpyDeviceToHost, s));
                    PJ_HIP(hipStreamSynchronize(s));
                }
            });
        } else {
            msbfs_solve(g, sources, n_src, dist_out);
        }
        g.have_result = false;  // g.dist does not hold a batch row
        g.batch_stats = true;
        return (int)PJ_OK;
    });
}

int pj_sssp_batch_write(pj_graph* pg, const int64_t* sources, int n_src, const char* const* paths, int strict) {
    if (!pg || (n_src > 0 && (!sources || !paths)) || n_src < 0) return arg_error("pj_sssp_batch_write: bad argument");
    for (int i = 0; i < n_src; ++i)
        if (!paths[i]) return arg_error("pj_sssp_batch_write: a path is NULL");
    return guarded([&] {
        Graph& g = pg->g;
        bind(*g.ctx);
        const size_t n = (size_t)g.n;
        std::atomic<int> err{PJ_OK};
        BatchWriter wr(n, paths, strict != 0, &err);
        if (g.weighted) {
            // concurrent solves (delta_batch); rows are gathered into host groups and written by the pool
            delta_batch(g, sources, n_src, g.batch_streams,
                        [&](int i, const int32_t* dev, hipStream_t s) { wr.add_row(i, dev, s); });
        } else {
            msbfs_each(g, sources, n_src, [&](int off, int ns, const int32_t* rows) {
                for (int k = 0; k < ns; ++k) wr.add_row(off + k, rows + (size_t)k * n);
            });
        }
        wr.finish();
        g.have_result = false;
        g.batch_stats = true;
        if (err.load() != PJ_OK) {
            set_error(wr.error());
            return err.load();
        }
        return (int)PJ_OK;
    });
}

int pj_last_stats(const pj_graph* pg, pj_stats* out) {
    if (!pg || !out) return arg_error("pj_last_stats: bad argument");
    if (!pg->g.have_result && !pg->g.batch_stats) {
        set_error("pj_last_stats: no solve has run on this graph");
        return PJ_ERR_STATE;
    }
    *out = pg->g.stats;
    return PJ_OK;
}

int pj_reach_stats(pj_graph* pg, pj_stats* out) {
    if (!pg) return arg_error("pj_reach_stats: graph is NULL");
    if (!pg->g.have_result) {
        set_error("pj_reach_stats: no solve has run on this graph");
        return PJ_ERR_STATE;
    }
    return guarded([&] {
        bind(*pg->g.ctx);
        i64 nr = 0, mr = 0;
        delta_materialize(pg->g);
        reach_stats(pg->g, &nr, &mr);
        pg->g.stats.reached = nr;
        pg->g.stats.reached_edges = mr;
        if (out) *out = pg->g.stats;
        return (int)PJ_OK;
    });
}

int pj_set_option(pj_graph* pg, const char* key, double value) {
    if (!pg || !key) return arg_error("pj_set_option: bad argument");
    Graph& g = pg->g;
    std::string k(key);
    if (k == "alpha" && value > 0) g.alpha = value;
    else if (k == "pull_vertex" && value >= 0) g.pull_vertex = value;
    else if (k == "beta" && value > 0) g.beta = value;
    else if (k == "delta" && value >= 0) g.delta = value;
    else if (k == "pull_factor" && value >= 0) g.pull_factor = value;
    else if (k == "defer_heavy" && value >= 0) g.defer_heavy = value;
    else if (k == "light_pull" && value >= 0) g.light_pull = value;
    else if (k == "tail_light_pull" && value > 0) g.tail_light_pull = value;
    else if (k == "round_log" && (value == 0 || value == 1)) g.round_log = (int)value;
    else if (k == "level_log" && (value == 0 || value == 1)) g.level_log = (int)value;
    else if (k == "spec_round" && (value == 0 || value == 1 || value == 2)) g.spec_round = (int)value;
    else if (k == "hub_first" && (value == 0 || value == 1)) g.hub_first = (int)value;
    else if (k == "pull_first" && (value == 0 || value == 1)) g.pull_first = (int)value;
    else if (k == "band_width" && value >= 0) g.band_width = value;
    else if (k == "tail_delta") g.tail_delta = value;
    else if (k == "tail_after" && value >= 0 && value < 1e6) g.tail_after = (int)value;
    else if (k == "tail_frac" && value >= 0) g.tail_frac = value;
    else if (k == "direction" && (value == 0 || value == 1 || value == 2)) g.force_mode = (int)value;
    else if (k == "level_batch" && value >= 0 && value <= 4096) g.level_batch = (int)value;
    else if (k == "round_batch" && value >= 1 && value <= 64) g.round_batch = (int)value;
    else if (k == "batch_streams" && value >= 1 && value <= 8) g.batch_streams = (int)value;
    else if (k == "light_filter" && (value == 0 || value == 1)) g.light_filter = (int)value;
    else if (k == "dense_frac" && value >= 0 && value <= 1) g.dense_frac = value;
    else if (k == "light_pack" && (value == 0 || value == 1)) g.light_pack = (int)value;
    else if (k == "split_w" && (value == 0 || value == 1)) g.split_w = (int)value;
    else if (k == "tail_pull" && (value == 0 || value == 1)) g.tail_pull = (int)value;
    else if (k == "spin_sync" && (value == 0 || value == 1)) g.spin_sync = (int)value;
    else if (k == "defer_check" && (value == 0 || value == 1)) g.defer_check = (int)value;
    else if (k == "round_gpc" && value >= 0 && value <= 64) g.round_gpc = (int)value;
    else if (k == "hub_gpc" && value >= 0 && value <= 64) g.hub_gpc = (int)value;
    else if (k == "heavy_gpc" && value >= 0 && value <= 64) g.heavy_gpc = (int)value;
    else if (k == "grid_per_cu" && value >= 0 && value <= 16) g.grid_per_cu = (int)value;
    else if (k == "max_levels" && value >= 0) g.max_levels = (int)value;
    else if (k == "bfs_small" && (value == 0 || value == 1)) g.bfs_small = (int)value;
    else if (k == "bfs_spare" && value >= 0 && value <= 16) g.bfs_spare = (int)value;
    else if (k == "ms_width" && (value == 0 || value == 1 || value == 2 || value == 4 || value == 8 || value == 16))
        g.ms_width = (int)value;
    else if (k == "ms_alpha" && value >= 0) g.ms_alpha = value;
    else if (k == "ms_streams" && value >= 1 && value <= 4) g.ms_streams = (int)value;
    else return arg_error("pj_set_option: unknown key or bad value");
    return PJ_OK;
}

// ------------------------------------------------------- binary CSR cache --
// Header + the device arrays in HBM order (pj.h). Streamed through one pinned
// staging buffer in 64 MiB pieces.

namespace {

struct CsrFileHeader {
    char magic[8];  // "PJCSR\0\0\1"
    uint32_t version;
    uint32_t flags;  // 1 weighted, 2 symmetric, 4 64-bit row offsets
    int64_t n, nnz;
    int64_t src_size, src_mtime_ns;
    uint64_t payload;  // bytes after the header
    uint64_t reserved;
};
static_assert(sizeof(CsrFileHeader) == 64, "header is 64 bytes");
constexpr char kCsrMagic[8] = {'P', 'J', 'C', 'S', 'R', 0, 0, 1};
constexpr size_t kStage = (size_t)64 << 20;

struct FileCloser {
    void operator()(FILE* f) const { if (f) std::fclose(f); }
};

void put_dev(FILE* f, const void* d, size_t bytes, PinnedBuf<char>& st, hipStream_t s) {
    for (size_t off = 0; off < bytes; off += kStage) {
        const size_t k = std::min(kStage, bytes - off);
        PJ_HIP(hipMemcpyAsync(st.p, static_cast<const char*>(d) + off, k, hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        if (std::fwrite(st.p, 1, k, f) != k) throw Error(PJ_ERR_IO, "pj_graph_save: write failed");
    }
}

void get_dev(FILE* f, void* d, size_t bytes, PinnedBuf<char>& st, hipStream_t s) {
    for (size_t off = 0; off < bytes; off += kStage) {
        const size_t k = std::min(kStage, bytes - off);
        if (std::fread(st.p, 1, k, f) != k) throw Error(PJ_ERR_PARSE, "pj_load_csr_file: file is truncated");
        PJ_HIP(hipMemcpyAsync(static_cast<char*>(d) + off, st.p, k, hipMemcpyHostToDevice, s));
        PJ_HIP(hipStreamSynchronize(s));
    }
}

uint64_t csr_payload(int64_t n, int64_t nnz, uint32_t flags) {
    const uint64_t ob = (flags & 4) ? 8 : 4;
    uint64_t b = ob * (uint64_t)(n + 1) + 4ull * (uint64_t)nnz;
    if (flags & 1) b += 4ull * (uint64_t)nnz;
    if (flags & 8) b += ob * (uint64_t)(n + 1) + 4ull * (uint64_t)nnz;  // the in-edge CSC
    return b;
}

}  // namespace

int pj_graph_save(const pj_graph* pg, const char* path, int64_t src_size, int64_t src_mtime_ns) {
    if (!pg || !path) return arg_error("pj_graph_save: bad argument");
    return guarded([&] {
        const Graph& g = pg->g;
        bind(*g.ctx);
        hipStream_t s = g.ctx->stream;
        CsrFileHeader h{};
        std::memcpy(h.magic, kCsrMagic, 8);
        h.version = 1;
        // flag 8: the CSC follows (unit-weight non-symmetric graphs; weighted graphs have none)
        const bool csc = !g.symmetric && !g.weighted;
        h.flags = (g.weighted ? 1u : 0u) | (g.symmetric ? 2u : 0u) | (g.off64 ? 4u : 0u) | (csc ? 8u : 0u);
        h.n = g.n;
        h.nnz = g.nnz;
        h.src_size = src_size;
        h.src_mtime_ns = src_mtime_ns;
        h.payload = csr_payload(g.n, g.nnz, h.flags);
        // write to a temporary name and rename, so a reader never sees a partial cache
        const std::string tmp = std::string(path) + ".tmp";
        std::unique_ptr<FILE, FileCloser> f(std::fopen(tmp.c_str(), "wb"));
        if (!f) {
            set_error(std::string("pj_graph_save: cannot open ") + tmp);
            return (int)PJ_ERR_IO;
        }
        if (std::fwrite(&h, sizeof h, 1, f.get()) != 1) throw Error(PJ_ERR_IO, "pj_graph_save: write failed");
        PinnedBuf<char> st;
        st.alloc(kStage);
        const size_t ob = g.off64 ? 8 : 4;
        put_dev(f.get(), g.row_ptr(), ob * (size_t)(g.n + 1), st, s);
        put_dev(f.get(), g.col.p, 4 * (size_t)g.nnz, st, s);
        if (g.weighted) put_dev(f.get(), g.w.p, 4 * (size_t)g.nnz, st, s);
        if (csc) {
            put_dev(f.get(), g.crow_ptr(), ob * (size_t)(g.n + 1), st, s);
            put_dev(f.get(), g.ccol.p, 4 * (size_t)g.nnz, st, s);
        }
        if (std::fclose(f.release()) != 0 || std::rename(tmp.c_str(), path) != 0) {
            std::remove(tmp.c_str());
            set_error(std::string("pj_graph_save: cannot write ") + path);
            return (int)PJ_ERR_IO;
        }
        return (int)PJ_OK;
    });
}

int pj_load_csr_file(pj_ctx* ctx, const char* path, int64_t expect_src_size, int64_t expect_src_mtime_ns,
                     pj_graph** out) {
    if (!ctx || !path || !out) return arg_error("pj_load_csr_file: bad argument");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        std::unique_ptr<FILE, FileCloser> f(std::fopen(path, "rb"));
        if (!f) {
            set_error(std::string("pj_load_csr_file: cannot open ") + path);
            return (int)PJ_ERR_IO;
        }
        CsrFileHeader h{};
        struct stat sb {};
        if (std::fread(&h, sizeof h, 1, f.get()) != 1 || std::memcmp(h.magic, kCsrMagic, 8) != 0 ||
            h.version != 1 || (h.flags & ~15u) != 0 || ((h.flags & 8) != 0) != ((h.flags & 3) == 0) || h.n < 0 || h.n > 0xFFFFFFFFll || h.nnz < 0 ||
            ((h.flags & 4) == 0 && (uint64_t)h.nnz > 0xFFFFFFFFull) ||
            h.payload != csr_payload(h.n, h.nnz, h.flags) || fstat(fileno(f.get()), &sb) != 0 ||
            (uint64_t)sb.st_size != sizeof h + h.payload) {
            set_error(std::string("pj_load_csr_file: not a libpj CSR file (or truncated): ") + path);
            return (int)PJ_ERR_PARSE;
        }
        if ((expect_src_size != -1 && expect_src_size != h.src_size) ||
            (expect_src_mtime_ns != -1 && expect_src_mtime_ns != h.src_mtime_ns)) {
            set_error(std::string("pj_load_csr_file: stale cache (source stamp differs): ") + path);
            return (int)PJ_ERR_STATE;
        }
        hipStream_t s = ctx->c.stream;
        auto pg = std::make_unique<pj_graph>();
        Graph& g = pg->g;
        g.ctx = &ctx->c;
        g.n = h.n;
        g.nnz = h.nnz;
        g.weighted = (h.flags & 1) != 0;
        g.symmetric = (h.flags & 2) != 0;
        g.off64 = (h.flags & 4) != 0;
        PinnedBuf<char> st;
        st.alloc(kStage);
        const size_t nr = (size_t)g.n + 1;
        if (g.off64) {
            g.row64.alloc(nr);
            get_dev(f.get(), g.row64.p, 8 * nr, st, s);
        } else {
            g.row32.alloc(nr);
            get_dev(f.get(), g.row32.p, 4 * nr, st, s);
        }
        g.col.alloc((size_t)g.nnz);
        get_dev(f.get(), g.col.p, 4 * (size_t)g.nnz, st, s);
        if (g.weighted) {
            g.w.alloc((size_t)g.nnz);
            get_dev(f.get(), g.w.p, 4 * (size_t)g.nnz, st, s);
        }
        if (h.flags & 8) {
            if (g.off64) {
                g.crow64.alloc(nr);
                get_dev(f.get(), g.crow64.p, 8 * nr, st, s);
            } else {
                g.crow32.alloc(nr);
                get_dev(f.get(), g.crow32.p, 4 * nr, st, s);
            }
            g.ccol.alloc((size_t)g.nnz);
            get_dev(f.get(), g.ccol.p, 4 * (size_t)g.nnz, st, s);
        }
        check_csr_device(g.row_ptr(), g.off64, g.col.p, g.n, g.nnz, s);
        if (h.flags & 8) check_csr_device(g.crow_ptr(), g.off64, g.ccol.p, g.n, g.nnz, s);
        return finish_graph(ctx, pg, out);
    });
}

int pj_load_snap_cached(pj_ctx* ctx, const char* path, int weighted, const char* cache_path, int write_back,
                        pj_graph** out) {
    if (!ctx || !path || !out) return arg_error("pj_load_snap_cached: bad argument");
    *out = nullptr;
    struct stat sb {};
    if (!cache_path || !*cache_path || stat(path, &sb) != 0) return pj_load_snap(ctx, path, weighted, out);
    const int64_t size = (int64_t)sb.st_size;
    const int64_t mtime = (int64_t)sb.st_mtim.tv_sec * 1000000000ll + (int64_t)sb.st_mtim.tv_nsec;
    if (pj_load_csr_file(ctx, cache_path, size, mtime, out) == PJ_OK) {
        if ((*out)->g.weighted == (weighted != 0)) return PJ_OK;
        pj_graph_destroy(*out);  // cached in the other weight mode: parse, and replace it
        *out = nullptr;
    }
    const int rc = pj_load_snap(ctx, path, weighted, out);
    if (rc == PJ_OK && write_back && pj_graph_save(*out, cache_path, size, mtime) != PJ_OK)
        fprintf(stderr, "warning: could not write the CSR cache %s: %s\n", cache_path, pj_last_error());
    return rc;
}

// ---------------------------------------------------------------- output --
// output_vector (:32-46): header line, then one decimal or "inf" per vertex.
// Formatting is split over host threads into per-chunk buffers and written
// in order, so the bytes are identical to the sequential writer.

static const char kHeader[] = "the vector is:\n";

int pj_format_sol(const int32_t* dist, int64_t n, char* buf, int64_t cap, int64_t* len_out) {
    if (n < 0 || (n > 0 && !dist) || !len_out) return arg_error("pj_format_sol: bad argument");
    std::vector<char> tmp((size_t)n * 12 + 16);
    size_t k = sizeof(kHeader) - 1;
    std::memcpy(tmp.data(), kHeader, k);
    k += format_rows(dist, 0, n, tmp.data() + k);
    *len_out = (int64_t)k;
    if (buf) {
        if (cap < (int64_t)k) return arg_error("pj_format_sol: buffer too small");
        std::memcpy(buf, tmp.data(), k);
    }
    return PJ_OK;
}

int pj_write_sol(const int32_t* dist, int64_t n, const char* path, int strict) {
    if (!path || n < 0 || (n > 0 && !dist)) return arg_error("pj_write_sol: bad argument");
    return guarded([&] {
        const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
        if (fd < 0) {
            if (strict) {
                set_error(std::string("cannot open ") + path);
                return (int)PJ_ERR_IO;
            }
            return (int)PJ_OK;  // the reference's ofstream fails silently (:617)
        }
        // batches of chunks: formatted in parallel, then written in parallel at their
        // offsets (pwrite), so the bytes equal the sequential writer's
        std::atomic<bool> ok{true};
        auto put = [&](const char* p, size_t len, int64_t off) {
            while (len) {
                const ssize_t r = pwrite(fd, p, len, (off_t)off);
                if (r <= 0) {
                    ok = false;
                    return;
                }
                p += r;
                len -= (size_t)r;
                off += r;
            }
        };
        put(kHeader, sizeof(kHeader) - 1, 0);
        int64_t pos = (int64_t)sizeof(kHeader) - 1;
        unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        const int64_t chunk = 1 << 18;
        const int64_t nchunks = (n + chunk - 1) / chunk;
        std::vector<std::vector<char>> out((size_t)std::min<int64_t>(nchunks, nt * 2));
        for (int64_t c0 = 0; c0 < nchunks; c0 += (int64_t)out.size()) {
            const int64_t cn = std::min<int64_t>((int64_t)out.size(), nchunks - c0);
            std::vector<size_t> lens((size_t)cn);
            std::vector<int64_t> offs((size_t)cn);
            std::vector<std::thread> th;
            for (int64_t c = 0; c < cn; ++c) {
                th.emplace_back([&, c] {
                    const int64_t a = (c0 + c) * chunk, b = std::min(n, a + chunk);
                    out[(size_t)c].resize((size_t)(b - a) * 12);
                    lens[(size_t)c] = format_rows(dist, a, b, out[(size_t)c].data());
                });
            }
            for (auto& t : th) t.join();
            th.clear();
            for (int64_t c = 0; c < cn; ++c) {
                offs[(size_t)c] = pos;
                pos += (int64_t)lens[(size_t)c];
            }
            for (int64_t c = 0; c < cn; ++c)
                th.emplace_back([&, c] { put(out[(size_t)c].data(), lens[(size_t)c], offs[(size_t)c]); });
            for (auto& t : th) t.join();
        }
        if (close(fd) != 0) ok = false;
        if (!ok && strict) {
            set_error(std::string("write failed: ") + path);
            return (int)PJ_ERR_IO;
        }
        return (int)PJ_OK;
    });
}

// ---- weighted SSSP over a 1D vertex partition (wpart.hip) -----------------

int pj_wpart_from_graph(pj_graph* g, int rank, int world, pj_wpart** out) {
    if (!g || !out) return arg_error("pj_wpart_from_graph: bad argument");
    if (world < 1 || world > 64 || rank < 0 || rank >= world)
        return arg_error("pj_wpart_from_graph: need 0 <= rank < world <= 64");
    *out = nullptr;
    return guarded([&] {
        bind(*g->g.ctx);
        *out = reinterpret_cast<pj_wpart*>(wpart_from_graph(g->g, rank, world));
        return (int)PJ_OK;
    });
}

int pj_wpart_generate_kronecker(pj_ctx* ctx, int scale, int edgefactor, uint64_t seed, int rank, int world,
                                pj_wpart** out) {
    if (!ctx || !out || scale < 0 || scale > 31 || edgefactor < 1 || edgefactor > 1024)
        return arg_error("pj_wpart_generate_kronecker: scale must be in [0,31], edgefactor in [1,1024]");
    if (world < 1 || world > 64 || rank < 0 || rank >= world)
        return arg_error("pj_wpart_generate_kronecker: need 0 <= rank < world <= 64");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        *out = reinterpret_cast<pj_wpart*>(wpart_from_kronecker(ctx->c, scale, edgefactor, seed, rank, world));
        return (int)PJ_OK;
    });
}

int pj_wpart_load_snap(pj_ctx* ctx, const char* path, int rank, int world, pj_wpart** out) {
    if (!ctx || !path || !out) return arg_error("pj_wpart_load_snap: bad argument");
    if (world < 1 || world > 64 || rank < 0 || rank >= world)
        return arg_error("pj_wpart_load_snap: need 0 <= rank < world <= 64");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        DevBuf<uint8_t> text;  // missing file: empty graph, as pj_load_snap (:67)
        const i64 len = read_file_to_device(ctx->c, path, text);
        DevBuf<u32> src, dst, w;
        ParseResult r = parse_device_text(ctx->c, text.p, len, true, src, dst, w);
        text.release();
        if (r.bad_line) {
            parse_error(r);
            return (int)PJ_ERR_PARSE;
        }
        *out = reinterpret_cast<pj_wpart*>(wpart_from_coo(ctx->c, src, dst, w, r.nnz, r.max_id + 1, rank, world));
        return (int)PJ_OK;
    });
}

int pj_wpart_load_snap_group(int world, pj_ctx* const* ctxs, const char* path, pj_wpart** out) {
    if (!ctxs || !path || !out || world < 1 || world > 64) return arg_error("pj_wpart_load_snap_group: bad argument");
    for (int r = 0; r < world; ++r) {
        if (!ctxs[r]) return arg_error("pj_wpart_load_snap_group: a context is NULL");
        out[r] = nullptr;
    }
    return guarded([&] {
        bind(ctxs[0]->c);
        DevBuf<uint8_t> text;  // missing file: empty graph, as pj_load_snap (:67)
        const i64 len = read_file_to_device(ctxs[0]->c, path, text);
        DevBuf<u32> src, dst, w;
        ParseResult r = parse_device_text(ctxs[0]->c, text.p, len, true, src, dst, w);
        text.release();
        if (r.bad_line) {
            parse_error(r);
            return (int)PJ_ERR_PARSE;
        }
        std::vector<Ctx*> cs;
        for (int k = 0; k < world; ++k) cs.push_back(&ctxs[k]->c);
        std::vector<WPart*> ps = wparts_from_coo_group(cs, src, dst, w, r.nnz, r.max_id + 1);
        for (int k = 0; k < world; ++k) out[k] = reinterpret_cast<pj_wpart*>(ps[(size_t)k]);
        bind(ctxs[0]->c);
        return (int)PJ_OK;
    });
}

int pj_wpart_destroy(pj_wpart* p) {
    if (!p) return PJ_OK;
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        delete_wpart(reinterpret_cast<WPart*>(p));
        return (int)PJ_OK;
    });
}

int pj_wpart_device_bytes(const pj_wpart* p, int64_t* out) {
    if (!p || !out) return arg_error("pj_wpart_device_bytes: bad argument");
    wpart_device_bytes(*reinterpret_cast<const WPart*>(p), out);
    return PJ_OK;
}

int pj_wpart_info(const pj_wpart* p, int64_t* out) {
    if (!p || !out) return arg_error("pj_wpart_info: bad argument");
    wpart_info(*reinterpret_cast<const WPart*>(p), out);
    return PJ_OK;
}

int pj_wpart_begin(pj_wpart* p, int64_t source, int32_t delta, int32_t* delta_out) {
    if (!p) return arg_error("pj_wpart_begin: bad argument");
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        const int32_t d = wpart_begin(*reinterpret_cast<WPart*>(p), source, delta);
        if (delta_out) *delta_out = d;
        return (int)PJ_OK;
    });
}

int pj_wpart_select(pj_wpart* p, int32_t lo, int32_t hi, int64_t* out) {
    if (!p || !out || lo < 0 || hi < lo) return arg_error("pj_wpart_select: bad argument");
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        wpart_select(*reinterpret_cast<WPart*>(p), lo, hi, out);
        return (int)PJ_OK;
    });
}

int pj_wpart_relax(pj_wpart* p, int light, int32_t lo, int32_t hi, uint64_t* send, int64_t* counts) {
    if (!p || !counts || lo < 0 || hi < lo) return arg_error("pj_wpart_relax: bad argument");
    return guarded([&] {
        WPart& P = *reinterpret_cast<WPart*>(p);
        // (the claim queue keeps one pair per improving remote relaxation, and an overflow rerun
        // re-sends from every band member: no bound known before the relax sizes a caller's
        // buffer, so the pairs are packed only into a buffer sized from the counts)
        if (send && wpart_world(P) > 1)
            throw Error(PJ_ERR_ARG, "pj_wpart_relax: pass send = NULL at world > 1, size the buffer from the counts "
                                    "and call pj_wpart_pack");
        bind(wpart_ctx(P));
        wpart_relax(P, light, lo, hi, counts);
        return (int)PJ_OK;
    });
}

int pj_wpart_pack(pj_wpart* p, uint64_t* send) {
    if (!p) return arg_error("pj_wpart_pack: bad argument");
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        WPart& P = *reinterpret_cast<WPart*>(p);
        if (!wpart_pending(P)) throw Error(PJ_ERR_STATE, "pj_wpart_pack: no relax is waiting to be packed");
        if (!send) throw Error(PJ_ERR_ARG, "pj_wpart_pack: send is NULL");
        wpart_pack(P, (u64*)send);
        return (int)PJ_OK;
    });
}

int pj_wpart_apply(pj_wpart* p, const uint64_t* recv, int64_t n_recv, int light, int32_t lo, int32_t hi) {
    if (!p || n_recv < 0 || (n_recv > 0 && !recv)) return arg_error("pj_wpart_apply: bad argument");
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        WPart& P = *reinterpret_cast<WPart*>(p);
        wpart_apply(P, (const u64*)recv, n_recv, light, lo, hi);
        PJ_HIP(hipStreamSynchronize(wpart_ctx(P).stream));  // the caller may reuse recv on return
        return (int)PJ_OK;
    });
}

int pj_wpart_end_round(pj_wpart* p, int64_t* n_f) {
    if (!p || !n_f) return arg_error("pj_wpart_end_round: bad argument");
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        *n_f = wpart_end_round(*reinterpret_cast<WPart*>(p));
        return (int)PJ_OK;
    });
}

int pj_wpart_reach(pj_wpart* p, int64_t* out) {
    if (!p || !out) return arg_error("pj_wpart_reach: bad argument");
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        wpart_reach(*reinterpret_cast<WPart*>(p), out);
        return (int)PJ_OK;
    });
}

int pj_wpart_copy_dist(pj_wpart* p, int32_t* dist_out) {
    if (!p || !dist_out) return arg_error("pj_wpart_copy_dist: bad argument");
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        wpart_copy_dist(*reinterpret_cast<WPart*>(p), dist_out);
        return (int)PJ_OK;
    });
}

// debug only (not declared in include/pj.h)
int pj_debug_bitmaps(pj_graph* pg, uint64_t* vis0, uint64_t* vis1, uint64_t* fnew) {
    if (!pg) return arg_error("pj_debug_bitmaps: graph is NULL");
    return guarded([&] {
        bind(*pg->g.ctx);
        debug_bitmaps(pg->g, (u64*)vis0, (u64*)vis1, (u64*)fnew);
        return (int)PJ_OK;
    });
}

// ---- 1D vertex partition (part.hip) ---------------------------------------

int pj_part_generate_kronecker(pj_ctx* ctx, int scale, int edgefactor, uint64_t seed, int rank, int world,
                               pj_part** out) {
    if (!ctx || !out || scale < 0 || scale > 31 || edgefactor < 1 || edgefactor > 1024)
        return arg_error("pj_part_generate_kronecker: scale must be in [0,31], edgefactor in [1,1024]");
    if (world < 1 || world > 64 || rank < 0 || rank >= world)
        return arg_error("pj_part_generate_kronecker: need 0 <= rank < world <= 64");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        *out = reinterpret_cast<pj_part*>(part_from_kronecker(ctx->c, scale, edgefactor, seed, rank, world));
        return (int)PJ_OK;
    });
}

int pj_part_load_coo(pj_ctx* ctx, const int64_t* src, const int64_t* dst, int64_t nnz, int64_t n_vertices,
                     int symmetric, int rank, int world, pj_part** out) {
    if (!ctx || !out || nnz < 0 || (nnz > 0 && (!src || !dst)))
        return arg_error("pj_part_load_coo: bad argument");
    if (world < 1 || world > 64 || rank < 0 || rank >= world)
        return arg_error("pj_part_load_coo: need 0 <= rank < world <= 64");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        i64 n = n_vertices;
        std::vector<u32> hs((size_t)nnz), hd((size_t)nnz);
        i64 mx = -1;
        for (i64 i = 0; i < nnz; ++i) {
            if (src[i] < 0 || dst[i] < 0 || src[i] > 0xFFFFFFFEll || dst[i] > 0xFFFFFFFEll)
                throw Error(PJ_ERR_RANGE, "pj_part_load_coo: id outside [0, 2^32-2]");
            mx = std::max(mx, std::max(src[i], dst[i]));
            hs[(size_t)i] = (u32)src[i];
            hd[(size_t)i] = (u32)dst[i];
        }
        if (n < 0) n = mx + 1;
        if (mx >= n) throw Error(PJ_ERR_RANGE, "pj_part_load_coo: id >= n_vertices");
        DevBuf<u32> s((size_t)nnz), d((size_t)nnz);
        if (nnz) {
            PJ_HIP(hipMemcpyAsync(s.p, hs.data(), sizeof(u32) * (size_t)nnz, hipMemcpyHostToDevice, ctx->c.stream));
            PJ_HIP(hipMemcpyAsync(d.p, hd.data(), sizeof(u32) * (size_t)nnz, hipMemcpyHostToDevice, ctx->c.stream));
            PJ_HIP(hipStreamSynchronize(ctx->c.stream));
        }
        *out = reinterpret_cast<pj_part*>(part_from_coo(ctx->c, s, d, nnz, n, rank, world, symmetric != 0));
        return (int)PJ_OK;
    });
}

int pj_part_load_snap(pj_ctx* ctx, const char* path, int rank, int world, pj_part** out) {
    if (!ctx || !path || !out) return arg_error("pj_part_load_snap: bad argument");
    if (world < 1 || world > 64 || rank < 0 || rank >= world)
        return arg_error("pj_part_load_snap: need 0 <= rank < world <= 64");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        DevBuf<uint8_t> text;  // missing file: empty graph, as pj_load_snap (:67)
        const i64 len = read_file_to_device(ctx->c, path, text);
        DevBuf<u32> src, dst, w;
        ParseResult r = parse_device_text(ctx->c, text.p, len, false, src, dst, w);
        text.release();
        if (r.bad_line) {
            parse_error(r);
            return (int)PJ_ERR_PARSE;
        }
        *out = reinterpret_cast<pj_part*>(part_from_coo(ctx->c, src, dst, r.nnz, r.max_id + 1, rank, world, false));
        return (int)PJ_OK;
    });
}

int pj_part_load_snap_group(int world, pj_ctx* const* ctxs, const char* path, pj_part** out) {
    if (!ctxs || !path || !out || world < 1 || world > 64) return arg_error("pj_part_load_snap_group: bad argument");
    for (int r = 0; r < world; ++r) {
        if (!ctxs[r]) return arg_error("pj_part_load_snap_group: a context is NULL");
        out[r] = nullptr;
    }
    return guarded([&] {
        bind(ctxs[0]->c);
        DevBuf<uint8_t> text;  // missing file: empty graph, as pj_load_snap (:67)
        const i64 len = read_file_to_device(ctxs[0]->c, path, text);
        DevBuf<u32> src, dst, w;
        ParseResult r = parse_device_text(ctxs[0]->c, text.p, len, false, src, dst, w);
        text.release();
        if (r.bad_line) {
            parse_error(r);
            return (int)PJ_ERR_PARSE;
        }
        std::vector<Ctx*> cs;
        for (int k = 0; k < world; ++k) cs.push_back(&ctxs[k]->c);
        std::vector<Part*> ps = parts_from_coo_group(cs, src, dst, r.nnz, r.max_id + 1, false);
        for (int k = 0; k < world; ++k) out[k] = reinterpret_cast<pj_part*>(ps[(size_t)k]);
        bind(ctxs[0]->c);
        return (int)PJ_OK;
    });
}

int pj_part_destroy(pj_part* p) {
    if (!p) return PJ_OK;
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        delete_part(reinterpret_cast<Part*>(p));
        return (int)PJ_OK;
    });
}

int pj_part_info_get(const pj_part* p, pj_part_info* out) {
    if (!p || !out) return arg_error("pj_part_info_get: bad argument");
    i64 v[25];
    part_info(*reinterpret_cast<const Part*>(p), v);
    out->n = v[0];
    out->lo = v[1];
    out->hi = v[2];
    out->block = v[3];
    out->words_per_rank = v[4];
    out->nnz_local = v[5];
    out->symmetric = (int32_t)v[6];
    out->off64 = (int32_t)v[7];
    out->rank = (int32_t)v[8];
    out->world = (int32_t)v[9];
    out->nnz_in_local = v[10];
    out->bytes_rows = v[11];
    out->bytes_state = v[12];
    out->bytes_bitmaps = v[13];
    out->bytes_exchange = v[14];
    for (int k = 0; k < 10; ++k) out->build_us[k] = v[15 + k];
    return PJ_OK;
}

int pj_part_zmask(pj_part* p, uint64_t* own_words) {
    if (!p || !own_words) return arg_error("pj_part_zmask: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        part_zmask(*reinterpret_cast<Part*>(p), reinterpret_cast<u64*>(own_words));
        return (int)PJ_OK;
    });
}

int pj_part_begin(pj_part* p, int64_t source, const uint64_t* iso, uint64_t* vis, int64_t* stats) {
    if (!p || !iso || !vis || !stats) return arg_error("pj_part_begin: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        part_begin(*reinterpret_cast<Part*>(p), source, reinterpret_cast<const u64*>(iso), reinterpret_cast<u64*>(vis),
                   stats);
        return (int)PJ_OK;
    });
}

int pj_part_push(pj_part* p, int level, uint64_t* vis, uint32_t* send, int64_t* counts) {
    if (!p || !vis || !counts || level < 0) return arg_error("pj_part_push: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        Part& P = *reinterpret_cast<Part*>(p);
        i64 info[25];
        part_info(P, info);
        if (info[9] > 1 && !send) throw Error(PJ_ERR_ARG, "pj_part_push: send is NULL");
        part_push(P, level, reinterpret_cast<u64*>(vis), send, counts);
        return (int)PJ_OK;
    });
}

int pj_part_apply(pj_part* p, int level, uint64_t* vis, const uint32_t* recv, int64_t n_recv) {
    if (!p || !vis || n_recv < 0 || (n_recv > 0 && !recv) || level < 0) return arg_error("pj_part_apply: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        part_apply(*reinterpret_cast<Part*>(p), level, reinterpret_cast<u64*>(vis), recv, n_recv);
        return (int)PJ_OK;
    });
}

int pj_part_pull(pj_part* p, int level, uint64_t* vis) {
    if (!p || !vis || level < 0) return arg_error("pj_part_pull: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        part_pull(*reinterpret_cast<Part*>(p), level, reinterpret_cast<u64*>(vis));
        return (int)PJ_OK;
    });
}

int pj_part_end_level(pj_part* p, uint64_t* vis, int64_t* stats) {
    if (!p || !vis || !stats) return arg_error("pj_part_end_level: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        part_end_level(*reinterpret_cast<Part*>(p), reinterpret_cast<u64*>(vis), stats);
        return (int)PJ_OK;
    });
}

int pj_part_reach(pj_part* p, int64_t* out) {
    if (!p || !out) return arg_error("pj_part_reach: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        part_reach(*reinterpret_cast<Part*>(p), out);
        return (int)PJ_OK;
    });
}

int pj_part_copy_dist(pj_part* p, int32_t* dist_out) {
    if (!p || !dist_out) return arg_error("pj_part_copy_dist: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        part_copy_dist(*reinterpret_cast<Part*>(p), dist_out);
        return (int)PJ_OK;
    });
}

const int32_t* pj_part_dist_device(pj_part* p) { return p ? part_dist_device(*reinterpret_cast<Part*>(p)) : nullptr; }

}  // extern "C"

// ---- transport and partitioned solves (comm.cpp, engine.cpp) ---------------

struct pj_comm {
    std::unique_ptr<pj::Comm> c;
};

namespace {

struct CallbackBfsSteps final : BfsSteps {
    pj_bfs_steps cb;
    explicit CallbackBfsSteps(const pj_bfs_steps& s) : cb(s) {
        n = s.n;
        nnz_local = s.nnz_local;
        bw = s.words_per_rank;
        block = s.block;
        rank = s.rank;
        world = s.world;
        vis = s.vis;
        iso = s.iso;
        zown = s.zown;
        send = s.send;
        recv = s.recv;
    }
    static void ok(int rc, const char* what) {
        if (rc != 0) throw Error(PJ_ERR_STATE, std::string("step callback ") + what + " failed");
    }
    void zmask() override { ok(cb.zmask(cb.user), "zmask"); }
    void begin(i64 source, i64* st3) override { ok(cb.begin(cb.user, source, st3), "begin"); }
    void push(int level, i64* counts) override { ok(cb.push(cb.user, level, counts), "push"); }
    void apply(int level, i64 nr) override { ok(cb.apply(cb.user, level, nr), "apply"); }
    void pull(int level) override { ok(cb.pull(cb.user, level), "pull"); }
    void end_level(i64* st3) override { ok(cb.end_level(cb.user, st3), "end_level"); }
};

struct CallbackDeltaSteps final : DeltaSteps {
    pj_delta_steps cb;
    explicit CallbackDeltaSteps(const pj_delta_steps& s) : cb(s) {
        n = s.n;
        rank = s.rank;
        world = s.world;
        send = s.send;
        recv = s.recv;
    }
    static void ok(int rc, const char* what) {
        if (rc != 0) throw Error(PJ_ERR_STATE, std::string("step callback ") + what + " failed");
    }
    int32_t begin(i64 source, int32_t delta) override {
        int32_t d = 0;
        ok(cb.begin(cb.user, source, delta, &d), "begin");
        return d;
    }
    void select(int32_t lo, int32_t hi, i64* out2) override { ok(cb.select(cb.user, lo, hi, out2), "select"); }
    void relax(int light, int32_t lo, int32_t hi, i64* counts) override {
        ok(cb.relax(cb.user, light, lo, hi, counts), "relax");
    }
    void apply(i64 nr, int light, int32_t lo, int32_t hi) override { ok(cb.apply(cb.user, nr, light, lo, hi), "apply"); }
    i64 end_round() override {
        int64_t nf = 0;
        ok(cb.end_round(cb.user, &nf), "end_round");
        return nf;
    }
    void reach(i64* out2) override { ok(cb.reach(cb.user, out2), "reach"); }
};

// Run fn(r) on one host thread per rank; the first failure's status and message win.
template <typename F>
int run_group(int world, F&& fn) {
    std::vector<int> rcs((size_t)world, PJ_OK);
    std::vector<std::string> msgs((size_t)world);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r)
        th.emplace_back([&, r] {
            rcs[(size_t)r] = guarded([&] { return fn(r); });
            if (rcs[(size_t)r] != PJ_OK) msgs[(size_t)r] = pj_last_error();
        });
    for (auto& t : th) t.join();
    // report the root cause, not a peer's "a peer rank failed"
    int first = -1;
    for (int r = 0; r < world; ++r)
        if (rcs[(size_t)r] != PJ_OK && (first < 0 || (rcs[(size_t)first] == PJ_ERR_COMM && rcs[(size_t)r] != PJ_ERR_COMM)))
            first = r;
    if (first < 0) return PJ_OK;
    set_error("rank " + std::to_string(first) + ": " + msgs[(size_t)first]);
    return rcs[(size_t)first];
}

// after a failed group solve (every rank thread joined): host groups are usable
// again; an aborted RCCL communicator stays unusable (pj_multi recreates its comms)
void reset_group(int world, pj_comm* const* comms) {
    for (int r = 0; r < world; ++r)
        if (comms[r]) comms[r]->c->reset();
}

}  // namespace

extern "C" {

int pj_comm_unique_id(uint8_t id[128]) {
    if (!id) return arg_error("pj_comm_unique_id: id is NULL");
    return guarded([&] {
        rccl_unique_id(id);
        return (int)PJ_OK;
    });
}

int pj_comm_create_rank(pj_ctx* ctx, int world, int rank, const uint8_t id[128], pj_comm** out) {
    if (!ctx || !out || world < 1 || rank < 0 || rank >= world || (world > 1 && !id))
        return arg_error("pj_comm_create_rank: bad argument");
    *out = nullptr;
    return guarded([&] {
        bind(ctx->c);
        auto c = std::make_unique<pj_comm>();
        // world 1 with an id is a one-rank RCCL group (exercises the RCCL calls)
        c->c = (world == 1 && !id) ? make_self_comm() : make_rccl_rank(ctx->c.device, world, rank, id);
        *out = c.release();
        return (int)PJ_OK;
    });
}

int pj_comm_create_group(pj_ctx* const* ctxs, int world, int transport, pj_comm** out) {
    if (!ctxs || !out || world < 1 || world > 64 || transport < 0 || transport > 2)
        return arg_error("pj_comm_create_group: bad argument");
    for (int r = 0; r < world; ++r) {
        if (!ctxs[r]) return arg_error("pj_comm_create_group: a ctx is NULL");
        out[r] = nullptr;
    }
    return guarded([&] {
        std::vector<int> dev;
        for (int r = 0; r < world; ++r) dev.push_back(ctxs[r]->c.device);
        std::vector<int> sorted = dev;
        std::sort(sorted.begin(), sorted.end());
        const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
        std::vector<std::unique_ptr<Comm>> cs;
        if (transport == PJ_TRANSPORT_RCCL || (transport == PJ_TRANSPORT_AUTO && distinct && world > 1))
            cs = make_rccl_group(dev);
        else if (world == 1) cs.push_back(make_self_comm());
        else cs = make_thread_comms(world, dev);
        for (int r = 0; r < world; ++r) {
            auto c = std::make_unique<pj_comm>();
            c->c = std::move(cs[(size_t)r]);
            out[r] = c.release();
        }
        return (int)PJ_OK;
    });
}

int pj_comm_create_callbacks(const pj_comm_callbacks* cb, pj_comm** out) {
    if (!cb || !out) return arg_error("pj_comm_create_callbacks: bad argument");
    *out = nullptr;
    return guarded([&] {
        auto c = std::make_unique<pj_comm>();
        c->c = make_callback_comm(*cb);
        *out = c.release();
        return (int)PJ_OK;
    });
}

int pj_comm_info(const pj_comm* c, int* rank, int* world, const char** kind) {
    if (!c) return arg_error("pj_comm_info: comm is NULL");
    if (rank) *rank = c->c->rank;
    if (world) *world = c->c->world;
    if (kind) *kind = c->c->kind();
    return PJ_OK;
}

int pj_comm_transport_ranks(const pj_comm* c, int* count, int* index) {
    if (!c || !count || !index) return arg_error("pj_comm_transport_ranks: bad argument");
    return guarded([&] {
        c->c->transport_ranks(count, index);
        return (int)PJ_OK;
    });
}

int pj_comm_destroy(pj_comm* c) {
    if (!c) return PJ_OK;
    return guarded([&] {
        delete c;
        return (int)PJ_OK;
    });
}

int pj_part_set_option(pj_part* p, const char* key, double value) {
    if (!p || !key) return arg_error("pj_part_set_option: bad argument");
    BfsParams& prm = part_params(*reinterpret_cast<Part*>(p));
    const std::string k(key);
    if (k == "alpha" && value > 0) prm.alpha = value;
    else if (k == "beta" && value > 0) prm.beta = value;
    else if (k == "direction" && (value == 0 || value == 1 || value == 2)) prm.force = (int)value;
    else if (k == "exchange_cap" && (value == -1 || value == 0 || value >= 64)) prm.xcap = (i64)value;
    else if (k == "single_gpu" && (value == 0 || value == 1))
        part_single_gpu(*reinterpret_cast<Part*>(p)) = (int)value;
    else return arg_error("pj_part_set_option: unknown key or bad value");
    return PJ_OK;
}

int pj_part_bfs(pj_part* p, pj_comm* comm, int64_t source, pj_part_stats* st) {
    if (!p || !comm) return arg_error("pj_part_bfs: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        Part& P = *reinterpret_cast<Part*>(p);
        if (part_single(P) && comm->c->world == 1) {
            part_solve_single(P, source, st);
            return (int)PJ_OK;
        }
        BfsSteps& S = part_steps(P);
        bool& iso = part_iso_ready(P, comm->c.get());
        bfs_engine(S, *comm->c, source, part_params(P), iso, st);
        iso = true;
        return (int)PJ_OK;
    });
}

int pj_part_bfs_group(int world, pj_part* const* parts, pj_comm* const* comms, int64_t source, pj_part_stats* st) {
    if (world < 1 || !parts || !comms) return arg_error("pj_part_bfs_group: bad argument");
    const int rc = run_group(world, [&](int r) { return pj_part_bfs(parts[r], comms[r], source, st ? st + r : nullptr); });
    if (rc != PJ_OK) reset_group(world, comms);
    return rc;
}

int pj_part_gather_dist(pj_part* p, pj_comm* comm, int32_t* dist_out) {
    if (!p || !comm) return arg_error("pj_part_gather_dist: bad argument");
    return guarded([&] {
        bind(part_ctx(*reinterpret_cast<Part*>(p)));
        part_gather_dist(*reinterpret_cast<Part*>(p), *comm->c, dist_out);
        return (int)PJ_OK;
    });
}

int pj_wpart_set_option(pj_wpart* p, const char* key, double value) {
    if (!p || !key) return arg_error("pj_wpart_set_option: bad argument");
    WPart& P = *reinterpret_cast<WPart*>(p);
    const std::string k(key);
    if (k == "tail_frac" && value >= 0) wpart_tail_params(P)[0] = value;
    else if (k == "tail_mult" && value >= 1) wpart_tail_params(P)[1] = value;
    else if (k == "pull_factor" && value >= 0) wpart_pull_factor(P) = value;
    else if (k == "light_pull" && value >= 0) wpart_light_pull(P) = value;
    else if (k == "tail_light_pull" && value >= 0) wpart_tail_light_pull(P) = value;
    else if (k == "single_gpu" && (value == 0 || value == 1)) wpart_single_gpu(P) = (int)value;
    else if (k == "pull_fmin" && (value == 0 || value == 1)) wpart_pull_fmin(P) = (int)value;
    else if (k == "grid_per_cu" && value >= 1 && value <= 32) wpart_grid_per_cu(P) = (int)value;
    else if (k == "queue_shard" && value >= 1 && value <= 1e9)
        return guarded([&] {
            bind(wpart_ctx(P));
            wpart_set_queue_shard(P, (i64)value);
            return (int)PJ_OK;
        });
    else return arg_error("pj_wpart_set_option: unknown key or bad value");
    return PJ_OK;
}

int pj_wpart_delta(pj_wpart* p, pj_comm* comm, int64_t source, int32_t delta, pj_part_stats* st) {
    if (!p || !comm) return arg_error("pj_wpart_delta: bad argument");
    return guarded([&] {
        WPart& P = *reinterpret_cast<WPart*>(p);
        bind(wpart_ctx(P));
        if (wpart_single(P) && comm->c->world == 1) wpart_solve_single(P, source, delta, st);
        else delta_engine(wpart_steps(P), *comm->c, source, delta, st);
        return (int)PJ_OK;
    });
}

int pj_wpart_delta_group(int world, pj_wpart* const* parts, pj_comm* const* comms, int64_t source, int32_t delta,
                         pj_part_stats* st) {
    if (world < 1 || !parts || !comms) return arg_error("pj_wpart_delta_group: bad argument");
    const int rc = run_group(
        world, [&](int r) { return pj_wpart_delta(parts[r], comms[r], source, delta, st ? st + r : nullptr); });
    if (rc != PJ_OK) reset_group(world, comms);
    return rc;
}

int pj_wpart_gather_dist(pj_wpart* p, pj_comm* comm, int32_t* dist_out) {
    if (!p || !comm) return arg_error("pj_wpart_gather_dist: bad argument");
    return guarded([&] {
        bind(wpart_ctx(*reinterpret_cast<WPart*>(p)));
        wpart_gather_dist(*reinterpret_cast<WPart*>(p), *comm->c, dist_out);
        return (int)PJ_OK;
    });
}

int pj_engine_bfs(const pj_bfs_steps* steps, pj_comm* comm, int64_t source, double alpha, double beta, int force,
                  pj_part_stats* st) {
    if (!steps || !comm || !steps->zmask || !steps->begin || !steps->push || !steps->apply || !steps->pull ||
        !steps->end_level || alpha <= 0 || beta <= 0 || force < 0 || force > 2)
        return arg_error("pj_engine_bfs: bad argument");
    return guarded([&] {
        CallbackBfsSteps S(*steps);
        BfsParams prm;
        prm.alpha = alpha;
        prm.beta = beta;
        prm.force = force;
        bfs_engine(S, *comm->c, source, prm, false, st);
        return (int)PJ_OK;
    });
}

int pj_engine_delta(const pj_delta_steps* steps, pj_comm* comm, int64_t source, int32_t delta, pj_part_stats* st) {
    if (!steps || !comm || !steps->begin || !steps->select || !steps->relax || !steps->apply || !steps->end_round ||
        !steps->reach)
        return arg_error("pj_engine_delta: bad argument");
    return guarded([&] {
        CallbackDeltaSteps S(*steps);
        delta_engine(S, *comm->c, source, delta, st);
        return (int)PJ_OK;
    });
}

}  // extern "C"
