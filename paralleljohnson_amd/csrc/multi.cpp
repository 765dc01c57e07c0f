// multi.cpp — the n-GPU handle of the C-ABI (SURVEY.md §8b `pj_create(int n_gpus, …)`):
// one call makes P ranks in this process (one pj_ctx and one host thread each,
// rank r on GPU r mod visible GPUs) and the transport between them, so a caller
// that ran `mpirun -np P parallel_johnson …` gets the same P-way run without a
// launcher. It is built only from the public entry points of pj.h:
//   - PJ_LAYOUT_PARTITIONED: the reference's 1D vertex partition (nn2rank
//     :169-200, every rank keeps its own rows instead of the scatter :344-410),
//     solved by the C++ protocol loops of engine.cpp over the pj_comm group
//     (exchange :522-554, termination :589-590), gathered like :612-614;
//   - PJ_LAYOUT_REPLICATED: every rank holds the whole graph and a batch of
//     sources is sharded over the ranks with no data-path collective (§8e.1).
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "internal.h"

struct pj_multi {
    int world = 0, transport = PJ_TRANSPORT_AUTO, layout = -1, weighted = 0;
    int ndev = 1;                  // visible GPUs (rank r runs on GPU r mod ndev)
    int64_t n = 0;
    std::vector<pj_ctx*> ctxs;
    std::vector<pj_comm*> comms;   // partitioned layout only
    std::vector<pj_part*> parts;   // partitioned, unit weights
    std::vector<pj_wpart*> wparts; // partitioned, weighted
    std::vector<pj_graph*> graphs; // replicated
    const char* kind = "none";
    std::string cache;             // CSR cache of replicated loads (pj_load_snap_cached)

    void drop_graph() {
        for (auto*& p : parts) pj_part_destroy(p), p = nullptr;
        for (auto*& p : wparts) pj_wpart_destroy(p), p = nullptr;
        for (auto*& g : graphs) pj_graph_destroy(g), g = nullptr;
        for (auto*& c : comms) pj_comm_destroy(c), c = nullptr;
        layout = -1;
        n = 0;
        kind = "none";
    }
};

namespace {

int arg_error(const char* msg) {
    pj::set_error(msg);
    return PJ_ERR_ARG;
}

// fn(r) on one host thread per rank; the root cause's status and message win over
// a peer's PJ_ERR_COMM ("a peer rank failed")
template <typename F>
int per_rank(int world, F&& fn) {
    std::vector<int> rcs((size_t)world, PJ_OK);
    std::vector<std::string> msgs((size_t)world);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r)
        th.emplace_back([&, r] {
            rcs[(size_t)r] = fn(r);
            if (rcs[(size_t)r] != PJ_OK) msgs[(size_t)r] = pj_last_error();
        });
    for (auto& t : th) t.join();
    int first = -1;
    for (int r = 0; r < world; ++r)
        if (rcs[(size_t)r] != PJ_OK && (first < 0 || (rcs[(size_t)first] == PJ_ERR_COMM && rcs[(size_t)r] != PJ_ERR_COMM)))
            first = r;
    if (first < 0) return PJ_OK;
    pj::set_error("rank " + std::to_string(first) + ": " + msgs[(size_t)first]);
    return rcs[(size_t)first];
}

// fn(r) for every rank of a replicated batch: one host thread per GPU, running the ranks that
// share it (world > visible GPUs) one after another. Each rank's batch fills the GPU by itself
// (its solves run on their own streams), so several host threads driving one GPU's batches
// gain nothing. (The intermittent illegal address test_multi_handle showed in round 6 was not
// this concurrency: it came back with the ranks in order, and was msbfs.hip's level ring
// running again past a pass's end on unwritten archive entries; see ms_live.) One rank per GPU
// (the product case) runs exactly as per_rank.
template <typename F>
int per_device(const pj_multi* m, F&& fn) {
    const int nd = std::max(1, std::min(m->ndev, m->world));
    std::vector<int> bad((size_t)nd, -1);
    const int rc = per_rank(nd, [&](int d) {
        for (int r = d; r < m->world; r += nd) {
            const int e = fn(r);
            if (e != PJ_OK) {
                bad[(size_t)d] = r;
                return e;
            }
        }
        return (int)PJ_OK;
    });
    if (rc != PJ_OK) {  // (per_rank named the failing thread; name the rank instead)
        std::string msg = pj_last_error();
        const size_t colon = msg.find(": ");
        if (msg.rfind("rank ", 0) == 0 && colon != std::string::npos) msg = msg.substr(colon + 2);
        for (int d = 0; d < nd; ++d)
            if (bad[(size_t)d] >= 0) {
                pj::set_error("rank " + std::to_string(bad[(size_t)d]) + ": " + msg);
                break;
            }
    }
    return rc;
}

int make_comms(pj_multi* m) {
    m->comms.assign((size_t)m->world, nullptr);
    const int rc = pj_comm_create_group(m->ctxs.data(), m->world, m->transport, m->comms.data());
    if (rc != PJ_OK) return rc;
    int rk = 0, w = 0;
    pj_comm_info(m->comms[0], &rk, &w, &m->kind);
    return PJ_OK;
}

// after a load: every rank agrees on n
int finish_load(pj_multi* m, int layout, int weighted) {
    m->layout = layout;
    m->weighted = weighted != 0;
    if (layout == PJ_LAYOUT_REPLICATED) {
        pj_graph_info(m->graphs[0], &m->n, nullptr, nullptr, nullptr);
        m->kind = "replicated";
    } else if (weighted) {
        int64_t info[8];
        pj_wpart_info(m->wparts[0], info);
        m->n = info[0];
    } else {
        pj_part_info pi{};
        pj_part_info_get(m->parts[0], &pi);
        m->n = pi.n;
    }
    return PJ_OK;
}

int check_loaded(const pj_multi* m, const char* who) {
    if (m->layout < 0) {
        pj::set_error(std::string(who) + ": no graph is loaded");
        return PJ_ERR_STATE;
    }
    return PJ_OK;
}

// one partitioned solve from `source`; dist_out (n int32, host) may be NULL
int part_solve(pj_multi* m, int64_t source, int32_t* dist_out, pj_part_stats* st) {
    std::vector<pj_part_stats> rs((size_t)m->world);
    int rc = m->weighted ? pj_wpart_delta_group(m->world, m->wparts.data(), m->comms.data(), source, 0, rs.data())
                         : pj_part_bfs_group(m->world, m->parts.data(), m->comms.data(), source, rs.data());
    if (rc != PJ_OK) {
        // a failed rank leaves an RCCL group aborted: recreate the comms so the handle
        // stays usable (host groups were reset by the group call); keep the first error
        const std::string err = pj_last_error();
        std::string kind(m->kind);
        if (kind == "rccl") {
            for (auto*& c : m->comms) pj_comm_destroy(c), c = nullptr;
            if (make_comms(m) != PJ_OK) m->drop_graph();  // unusable: the caller must load again
        }
        pj::set_error(err);
        return rc;
    }
    if (st) {  // the reference's Time: is rank 0's clock after the last round (:597-605); max over ranks here
        *st = rs[0];
        for (auto& s : rs) st->solve_ms = std::max(st->solve_ms, s.solve_ms);
    }
    return per_rank(m->world, [&](int r) {  // MPI_Gatherv :612-614
        int32_t* o = r == 0 ? dist_out : nullptr;
        return m->weighted ? pj_wpart_gather_dist(m->wparts[(size_t)r], m->comms[(size_t)r], o)
                           : pj_part_gather_dist(m->parts[(size_t)r], m->comms[(size_t)r], o);
    });
}

}  // namespace

extern "C" {

int pj_multi_create(int n_gpus, int transport, pj_multi** out) {
    if (!out || n_gpus < 1 || transport < PJ_TRANSPORT_AUTO || transport > PJ_TRANSPORT_HOST)
        return arg_error("pj_multi_create: bad argument");
    *out = nullptr;
    int ndev = 0;
    pj_device_count(&ndev);
    if (ndev < 1) {
        pj::set_error("pj_multi_create: no HIP device visible");
        return PJ_ERR_HIP;
    }
    auto* m = new pj_multi;
    m->world = n_gpus;
    m->ndev = ndev;
    m->transport = transport;
    m->ctxs.assign((size_t)n_gpus, nullptr);
    for (int r = 0; r < n_gpus; ++r) {
        const int rc = pj_create(r % ndev, &m->ctxs[(size_t)r]);
        if (rc != PJ_OK) {
            pj_multi_destroy(m);
            return rc;
        }
    }
    *out = m;
    return PJ_OK;
}

int pj_multi_destroy(pj_multi* m) {
    if (!m) return PJ_OK;
    m->drop_graph();
    for (auto* c : m->ctxs) pj_destroy(c);
    delete m;
    return PJ_OK;
}

int pj_multi_ctx(pj_multi* m, int rank, pj_ctx** out) {
    if (!m || !out || rank < 0 || rank >= m->world) return arg_error("pj_multi_ctx: bad argument");
    *out = m->ctxs[(size_t)rank];
    return PJ_OK;
}

int pj_multi_set_csr_cache(pj_multi* m, const char* cache_path) {
    if (!m) return arg_error("pj_multi_set_csr_cache: bad argument");
    m->cache = cache_path ? cache_path : "";
    return PJ_OK;
}

int pj_multi_load_snap(pj_multi* m, const char* path, int weighted, int layout) {
    if (!m || !path || (layout != PJ_LAYOUT_PARTITIONED && layout != PJ_LAYOUT_REPLICATED))
        return arg_error("pj_multi_load_snap: bad argument");
    m->drop_graph();
    const int P = m->world;
    int rc;
    if (layout == PJ_LAYOUT_REPLICATED) {
        m->graphs.assign((size_t)P, nullptr);
        // rank 0 alone writes the cache when it is missing or stale
        rc = per_rank(P, [&](int r) {
            return pj_load_snap_cached(m->ctxs[(size_t)r], path, weighted, m->cache.empty() ? nullptr : m->cache.c_str(),
                                       r == 0, &m->graphs[(size_t)r]);
        });
    } else {
        rc = make_comms(m);
        if (rc == PJ_OK) {
            m->parts.assign((size_t)P, nullptr);
            m->wparts.assign((size_t)P, nullptr);
            // one parse on rank 0's GPU, each rank's entries scattered to it (:313-338, :344-410)
            rc = weighted ? pj_wpart_load_snap_group(P, m->ctxs.data(), path, m->wparts.data())
                          : pj_part_load_snap_group(P, m->ctxs.data(), path, m->parts.data());
        }
    }
    if (rc != PJ_OK) {
        const std::string msg = pj_last_error();
        m->drop_graph();
        pj::set_error(msg);
        return rc;
    }
    return finish_load(m, layout, weighted);
}

int pj_multi_generate_kronecker(pj_multi* m, int scale, int edgefactor, uint64_t seed, int weighted, int layout) {
    if (!m || (layout != PJ_LAYOUT_PARTITIONED && layout != PJ_LAYOUT_REPLICATED))
        return arg_error("pj_multi_generate_kronecker: bad argument");
    m->drop_graph();
    const int P = m->world;
    int rc;
    if (layout == PJ_LAYOUT_REPLICATED) {
        m->graphs.assign((size_t)P, nullptr);
        rc = per_rank(P, [&](int r) {
            return pj_generate_kronecker(m->ctxs[(size_t)r], scale, edgefactor, seed, weighted, &m->graphs[(size_t)r]);
        });
    } else {
        rc = make_comms(m);
        if (rc == PJ_OK) {
            m->parts.assign((size_t)P, nullptr);
            m->wparts.assign((size_t)P, nullptr);
            rc = per_rank(P, [&](int r) {  // every rank enumerates the tuples and keeps its block's rows
                return weighted ? pj_wpart_generate_kronecker(m->ctxs[(size_t)r], scale, edgefactor, seed, r, P,
                                                              &m->wparts[(size_t)r])
                                : pj_part_generate_kronecker(m->ctxs[(size_t)r], scale, edgefactor, seed, r, P,
                                                             &m->parts[(size_t)r]);
            });
        }
    }
    if (rc != PJ_OK) {
        const std::string msg = pj_last_error();
        m->drop_graph();
        pj::set_error(msg);
        return rc;
    }
    return finish_load(m, layout, weighted);
}

int pj_multi_device_bytes(const pj_multi* m, int rank, int64_t* out) {
    if (!m || !out || rank < 0 || rank >= m->world) return arg_error("pj_multi_device_bytes: bad argument");
    const int rc = check_loaded(m, "pj_multi_device_bytes");
    if (rc != PJ_OK) return rc;
    for (int k = 0; k < 4; ++k) out[k] = 0;
    if (m->layout == PJ_LAYOUT_REPLICATED) {
        int64_t n = 0, nnz = 0;
        int32_t w = 0, sym = 0;
        pj_graph_info(m->graphs[(size_t)rank], &n, &nnz, &w, &sym);
        out[0] = 4 * (n + 1) + (4 + (w ? 4 : 0)) * nnz;  // (row offsets, columns, weights)
        return PJ_OK;
    }
    if (m->weighted) return pj_wpart_device_bytes(m->wparts[(size_t)rank], out);
    pj_part_info pi{};
    const int e = pj_part_info_get(m->parts[(size_t)rank], &pi);
    out[0] = pi.bytes_rows;
    out[1] = pi.bytes_state;
    out[2] = pi.bytes_bitmaps;
    out[3] = pi.bytes_exchange;
    return e;
}

int pj_multi_info(const pj_multi* m, pj_multi_info_t* out) {
    if (!m || !out) return arg_error("pj_multi_info: bad argument");
    out->n = m->n;
    out->world = m->world;
    out->layout = m->layout;
    out->weighted = m->weighted;
    out->transport = m->kind;
    return PJ_OK;
}

int pj_multi_sssp(pj_multi* m, int64_t source, int32_t* dist_out, pj_part_stats* st) {
    if (!m) return arg_error("pj_multi_sssp: bad argument");
    if (int rc = check_loaded(m, "pj_multi_sssp")) return rc;
    if (m->layout == PJ_LAYOUT_PARTITIONED) return part_solve(m, source, dist_out, st);
    // replicated: one GPU answers a single source
    pj_graph* g = m->graphs[0];
    int rc = pj_sssp(g, source, dist_out);
    if (rc == PJ_OK && st) {
        pj_stats s{};
        pj_last_stats(g, &s);
        *st = pj_part_stats{};
        st->solve_ms = s.kernel_ms;
        st->levels = s.levels;
        st->td_levels = s.td_levels;
        st->bu_levels = s.bu_levels;
        if (pj_reach_stats(g, &s) != PJ_OK) return PJ_ERR_STATE;
        st->reached = s.reached;
        st->reached_edges = s.reached_edges;
    }
    return rc;
}

int pj_multi_sssp_batch_write(pj_multi* m, const int64_t* sources, int n_src, const char* const* paths, int strict,
                              double* solve_ms) {
    if (!m || n_src < 0 || (n_src > 0 && (!sources || !paths))) return arg_error("pj_multi_sssp_batch_write: bad argument");
    for (int i = 0; i < n_src; ++i)
        if (!paths[i]) return arg_error("pj_multi_sssp_batch_write: a path is NULL");
    if (int rc = check_loaded(m, "pj_multi_sssp_batch_write")) return rc;
    const int P = m->world;
    if (m->layout == PJ_LAYOUT_PARTITIONED) {  // one partitioned solve per source
        std::vector<int32_t> dist((size_t)m->n);
        double t = 0;
        for (int i = 0; i < n_src; ++i) {
            pj_part_stats st{};
            int rc = part_solve(m, sources[i], dist.data(), &st);
            if (rc == PJ_OK) rc = pj_write_sol(dist.data(), m->n, paths[i], strict);
            if (rc != PJ_OK) return rc;
            t += st.solve_ms;
        }
        if (solve_ms) *solve_ms = t;
        return PJ_OK;
    }
    // replicated: rank r takes sources r, r + P, ... and writes their files
    std::vector<double> kms((size_t)P, 0.0);
    const int rc = per_device(m, [&](int r) {
        std::vector<int64_t> mine;
        std::vector<const char*> pp;
        for (int i = r; i < n_src; i += P) {
            mine.push_back(sources[i]);
            pp.push_back(paths[i]);
        }
        if (mine.empty()) return (int)PJ_OK;
        int e = pj_sssp_batch_write(m->graphs[(size_t)r], mine.data(), (int)mine.size(), pp.data(), strict);
        pj_stats st{};
        if (e == PJ_OK && pj_last_stats(m->graphs[(size_t)r], &st) == PJ_OK) kms[(size_t)r] = st.kernel_ms;
        return e;
    });
    if (rc == PJ_OK && solve_ms) *solve_ms = *std::max_element(kms.begin(), kms.end());
    return rc;
}

int pj_multi_sssp_batch(pj_multi* m, const int64_t* sources, int n_src, int32_t* dist_out) {
    if (!m || n_src < 0 || (n_src > 0 && !sources)) return arg_error("pj_multi_sssp_batch: bad argument");
    if (int rc = check_loaded(m, "pj_multi_sssp_batch")) return rc;
    const size_t n = (size_t)m->n;
    if (m->layout == PJ_LAYOUT_PARTITIONED) {
        for (int i = 0; i < n_src; ++i)
            if (int rc = part_solve(m, sources[i], dist_out ? dist_out + (size_t)i * n : nullptr, nullptr)) return rc;
        return PJ_OK;
    }
    const int P = m->world;
    return per_device(m, [&](int r) {
        std::vector<int64_t> mine;
        for (int i = r; i < n_src; i += P) mine.push_back(sources[i]);
        if (mine.empty()) return (int)PJ_OK;
        std::vector<int32_t> rows(dist_out ? mine.size() * n : 0);
        int e = pj_sssp_batch(m->graphs[(size_t)r], mine.data(), (int)mine.size(), dist_out ? rows.data() : nullptr);
        if (e == PJ_OK && dist_out)
            for (size_t k = 0; k < mine.size(); ++k)
                std::copy(rows.begin() + k * n, rows.begin() + (k + 1) * n, dist_out + (size_t)(r + (int)k * P) * n);
        return e;
    });
}

}  // extern "C"
