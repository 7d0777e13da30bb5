// mspmv_dist.hip -- row-block sharded SpMM and block CG over several GPUs (include/mspmv_dist.h).
// Host planning is plain C++ (testable without a GPU); the data path is HIP kernels on the
// local handle's stream plus RCCL point-to-point halo exchange and all-reduces over xGMI.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mspmv_dist.h"
#include "mspmv_internal.h"

using namespace mspmv;

namespace {

mspmv_status fail_msg(mspmv_status st, const std::string &msg)
{
    set_error(msg);
    return st;
}

#define D_HIP(expr)                                                                                \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return fail_msg(_e == hipErrorOutOfMemory ? MSPMV_ERR_OOM : MSPMV_ERR_HIP,             \
                            std::string(#expr) + ": " + hipGetErrorString(_e));                    \
    } while (0)

#define D_NCCL(expr)                                                                               \
    do {                                                                                           \
        ncclResult_t _r = (expr);                                                                  \
        if (_r != ncclSuccess)                                                                     \
            return fail_msg(MSPMV_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(_r));   \
    } while (0)

#define D_ST(expr)                                                                                 \
    do {                                                                                           \
        mspmv_status _s = (expr);                                                                  \
        if (_s != MSPMV_OK)                                                                        \
            return _s;                                                                             \
    } while (0)

template <typename T>
mspmv_status dalloc(T **p, size_t n)
{
    *p = nullptr;
    hipError_t e = hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        return fail_msg(e == hipErrorOutOfMemory ? MSPMV_ERR_OOM : MSPMV_ERR_HIP,
                        std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    return MSPMV_OK;
}

template <typename T>
void dfree(T *&p)
{
    if (p)
        (void)hipFree((void *)p);
    p = nullptr;
}

}  // namespace

// One per rank: the RCCL communicator and the one stream every collective of every sharded object
// on this rank is enqueued on (the objects' local handles run on it too).  All collectives of a rank
// then form a single stream-ordered sequence, issued by one host thread in the program's order, so
// every rank meets them in the same order and no two communicators can ever have collectives in
// flight at once (RCCL/NCCL: concurrent operations on different communicators may deadlock).
struct mspmv_comm_s {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;
    int users = 0;  // sharded objects created on it (mspmv_comm_destroy refuses while > 0)
};

struct mspmv_dist_s {
    mspmv_comm_s *cm = nullptr;
    bool own_cm = false;  // mspmv_dist_create: a private communicator, destroyed with the object
    ncclComm_t comm = nullptr;  // == cm->comm
    int nranks = 1, rank = 0, device = 0;
    int row_lo = 0, n_own = 0, n_halo = 0, n_send = 0;
    std::vector<int> row_begin;
    mspmv_handle local = nullptr;  // n_own x (n_own + n_halo) local CSR, owns the stream
    // exchange plan (element counts in rows; multiplied by L at run time)
    std::vector<int> send_counts, send_displs, recv_counts, recv_displs;
    int *d_send_idx = nullptr;  // owned row index of every row to send, grouped by peer
    // buffers (grown to the largest L used)
    int cap_L = 0;
    double *d_pext = nullptr;   // (n_own + n_halo) x L : [p_own | p_halo]
    double *d_send = nullptr;   // n_send x L
    double *d_r = nullptr, *d_ap = nullptr;  // n_own x L
    double *d_partials = nullptr;
    size_t partials_cap = 0;
    unsigned *d_gtickets = nullptr;
    size_t gtickets_cap = 0;
    CgScalars *d_scal = nullptr;
    unsigned char *d_conv = nullptr;
    CgControl *d_ctrl = nullptr;
    CgControl *h_ctrl = nullptr;  // pinned
    double *d_red = nullptr;      // [2 L]: p.Ap, r.r
    double *d_hist = nullptr;
    int hist_cap = 0;
    // SpMM overlap (mspmv_dist_spmm_dev): the local rows split into [0, int_lo) | [int_lo, int_hi)
    // | [int_hi, n_own), the middle range referencing owned columns only.  The middle runs on its
    // own handle's stream while `local`'s stream packs and exchanges the halo; head and tail
    // follow the exchange.  Null handles when the split does not pay (no interior worth it).
    mspmv_handle part[3] = {nullptr, nullptr, nullptr};
    int int_lo = 0, int_hi = 0;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // x ready, mid, halo, head, tail
    // CG: K iterations (kernels, the interior's second stream, the RCCL exchange and all-reduces)
    // captured once into a graph and replayed per batch while the key (buffers, plans, L, tolerance,
    // history size, K) is unchanged.  Captured only after one eager batch has run on this object,
    // so RCCL has set up its connections outside the capture.
    hipGraph_t cg_graph = nullptr;
    hipGraphExec_t cg_exec = nullptr;
    std::vector<const void *> cg_key;
    bool cg_warm = false;
    // test hook (mspmv_dist_test_poison_tickets): the next CG solve's fold tickets start dirty
    unsigned poison_value = 0;
    int poison_flags = 0;
};

extern "C" {

mspmv_status mspmv_dist_partition(const int *row_offsets, int num_rows, int num_nonzeros, int nranks, int *row_begin)
{
    if (!row_offsets || !row_begin || nranks < 1 || num_rows < 0 || num_nonzeros < 0)
        return fail_msg(MSPMV_ERR_INVALID, "dist_partition: bad arguments");
    const long long total = (long long)num_rows + num_nonzeros;
    const long long step = (total + nranks - 1) / nranks;
    const int *a = row_offsets + 1;
    for (int g = 0; g <= nranks; ++g) {
        const long long dl = std::min(step * g, total);
        const int d = (int)dl;
        int lo = std::max(d - num_nonzeros, 0), hi = std::min(d, num_rows);
        while (lo < hi) {
            const int pivot = (lo + hi) >> 1;
            if (a[pivot] <= d - pivot - 1)
                lo = pivot + 1;
            else
                hi = pivot;
        }
        row_begin[g] = std::min(lo, num_rows);
    }
    row_begin[0] = 0;
    row_begin[nranks] = num_rows;
    return MSPMV_OK;
}

mspmv_status mspmv_dist_localize(const int *row_begin, int nranks, int rank, const int *local_row_offsets,
                                 const int *global_cols, int *local_cols, int *n_halo, int *halo_global, int halo_cap,
                                 int *halo_counts)
{
    if (!row_begin || nranks < 1 || rank < 0 || rank >= nranks || !local_row_offsets || !n_halo)
        return fail_msg(MSPMV_ERR_INVALID, "dist_localize: bad arguments");
    const int lo = row_begin[rank], hi = row_begin[rank + 1];
    const int rows = hi - lo;
    const int nnz = local_row_offsets[rows];
    if (nnz > 0 && !global_cols)
        return fail_msg(MSPMV_ERR_INVALID, "dist_localize: null columns");
    std::vector<int> halo;
    halo.reserve(1024);
    for (int k = 0; k < nnz; ++k) {
        const int c = global_cols[k];
        if (c < lo || c >= hi)
            halo.push_back(c);
    }
    std::sort(halo.begin(), halo.end());
    halo.erase(std::unique(halo.begin(), halo.end()), halo.end());
    *n_halo = (int)halo.size();
    if (halo_counts) {
        for (int g = 0; g < nranks; ++g) {
            auto b = std::lower_bound(halo.begin(), halo.end(), row_begin[g]);
            auto e = std::lower_bound(halo.begin(), halo.end(), row_begin[g + 1]);
            halo_counts[g] = (int)(e - b);
        }
    }
    if (halo_global) {
        if (halo_cap < (int)halo.size())
            return fail_msg(MSPMV_ERR_INVALID, "dist_localize: halo_cap too small");
        std::copy(halo.begin(), halo.end(), halo_global);
    }
    if (local_cols) {
        const int n_own = rows;
#pragma omp parallel for schedule(static)
        for (int k = 0; k < nnz; ++k) {
            const int c = global_cols[k];
            if (c >= lo && c < hi)
                local_cols[k] = c - lo;
            else
                local_cols[k] = n_own + (int)(std::lower_bound(halo.begin(), halo.end(), c) - halo.begin());
        }
    }
    return MSPMV_OK;
}

mspmv_status mspmv_comm_unique_id(unsigned char id[MSPMV_UNIQUE_ID_BYTES])
{
    static_assert(sizeof(ncclUniqueId) == MSPMV_UNIQUE_ID_BYTES, "RCCL unique id size");
    if (!id)
        return fail_msg(MSPMV_ERR_INVALID, "null id");
    ncclUniqueId u;
    D_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return MSPMV_OK;
}

mspmv_status mspmv_dist_destroy(mspmv_dist d)
{
    if (!d)
        return MSPMV_OK;
    (void)hipSetDevice(d->device);
    if (d->local)
        mspmv_sync(d->local);
    dfree(d->d_send_idx);
    dfree(d->d_pext);
    dfree(d->d_send);
    dfree(d->d_r);
    dfree(d->d_ap);
    dfree(d->d_partials);
    dfree(d->d_gtickets);
    dfree(d->d_scal);
    dfree(d->d_conv);
    dfree(d->d_ctrl);
    dfree(d->d_red);
    dfree(d->d_hist);
    if (d->h_ctrl)
        (void)hipHostFree(d->h_ctrl);
    if (d->cg_exec)
        (void)hipGraphExecDestroy(d->cg_exec);
    if (d->cg_graph)
        (void)hipGraphDestroy(d->cg_graph);
    for (auto &ph : d->part)
        if (ph)
            mspmv_destroy(ph);
    for (auto &e : d->ev)
        if (e)
            (void)hipEventDestroy(e);
    if (d->local)
        mspmv_destroy(d->local);
    if (d->cm) {
        --d->cm->users;
        if (d->own_cm)
            mspmv_comm_destroy(d->cm);
    }
    delete d;
    return MSPMV_OK;
}

mspmv_status mspmv_comm_create(const unsigned char id[MSPMV_UNIQUE_ID_BYTES], int nranks, int rank, int device,
                               mspmv_comm *out)
{
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return fail_msg(MSPMV_ERR_INVALID, "comm_create: bad arguments");
    *out = nullptr;
    D_HIP(hipSetDevice(device));
    auto *c = new mspmv_comm_s();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail_msg(MSPMV_ERR_HIP, "comm_create: hipStreamCreate failed");
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t nr = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (nr != ncclSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return fail_msg(MSPMV_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(nr));
    }
    *out = c;
    return MSPMV_OK;
}

mspmv_status mspmv_comm_destroy(mspmv_comm c)
{
    if (!c)
        return MSPMV_OK;
    if (c->users > 0)
        return fail_msg(MSPMV_ERR_INVALID, "comm_destroy: sharded objects still use this communicator");
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->comm)
        ncclCommDestroy(c->comm);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return MSPMV_OK;
}

mspmv_status mspmv_dist_create(const unsigned char id[MSPMV_UNIQUE_ID_BYTES], int nranks, int rank, int device,
                               const int *row_begin, const mspmv_csr_d *local_rows, mspmv_dist *out)
{
    if (!id || !row_begin || !local_rows || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return fail_msg(MSPMV_ERR_INVALID, "dist_create: bad arguments");
    *out = nullptr;
    mspmv_comm c = nullptr;
    D_ST(mspmv_comm_create(id, nranks, rank, device, &c));
    mspmv_dist d = nullptr;
    const mspmv_status st = mspmv_dist_create_on(c, row_begin, local_rows, &d);
    if (st != MSPMV_OK) {
        mspmv_comm_destroy(c);
        return st;
    }
    d->own_cm = true;
    *out = d;
    return MSPMV_OK;
}

mspmv_status mspmv_dist_create_on(mspmv_comm c, const int *row_begin, const mspmv_csr_d *local_rows,
                                  mspmv_dist *out)
{
    if (!c || !row_begin || !local_rows || !out)
        return fail_msg(MSPMV_ERR_INVALID, "dist_create: bad arguments");
    *out = nullptr;
    const int nranks = c->nranks, rank = c->rank, device = c->device;
    const int lo = row_begin[rank], hi = row_begin[rank + 1];
    if (local_rows->num_rows != hi - lo || local_rows->num_cols != row_begin[nranks])
        return fail_msg(MSPMV_ERR_INVALID, "dist_create: local rows do not match row_begin (square matrix needed)");
    D_HIP(hipSetDevice(device));
    auto *d = new mspmv_dist_s();
    d->cm = c;
    ++c->users;
    d->comm = c->comm;
    d->nranks = nranks;
    d->rank = rank;
    d->device = device;
    d->row_lo = lo;
    d->n_own = hi - lo;
    d->row_begin.assign(row_begin, row_begin + nranks + 1);
    auto bail = [&](mspmv_status s) {
        mspmv_dist_destroy(d);
        return s;
    };
    ncclResult_t nr = ncclSuccess;
    // localize this rank's rows
    const int nnz = local_rows->num_nonzeros;
    std::vector<int> lcols((size_t)std::max(nnz, 1));
    std::vector<int> halo_counts(nranks);
    int n_halo = 0;
    mspmv_status st = mspmv_dist_localize(row_begin, nranks, rank, local_rows->row_offsets, local_rows->column_indices,
                                          nullptr, &n_halo, nullptr, 0, nullptr);
    if (st != MSPMV_OK)
        return bail(st);
    std::vector<int> halo((size_t)std::max(n_halo, 1));
    st = mspmv_dist_localize(row_begin, nranks, rank, local_rows->row_offsets, local_rows->column_indices,
                             lcols.data(), &n_halo, halo.data(), n_halo, halo_counts.data());
    if (st != MSPMV_OK)
        return bail(st);
    d->n_halo = n_halo;
    mspmv_csr_d lc = *local_rows;
    lc.num_cols = d->n_own + n_halo;
    lc.column_indices = lcols.data();
    // the local handle runs on the communicator's stream: this object's kernels and collectives, and
    // every other object's on this rank, are one stream-ordered sequence
    if ((st = csr_create_on_stream(&lc, device, c->stream, &d->local)) != MSPMV_OK)
        return bail(st);
    // interior rows: the longest contiguous run of rows that reference owned columns only (for a
    // banded / FEM matrix cut into row blocks, everything but the rows within the band of either
    // block end); split off only when it holds >= half the nonzeros and there is a halo at all
    // MSPMV_DIST_FORCE_SPLIT=1 (tests): split at the row thirds even without a halo, so one GPU
    // exercises the three-stream path (RCCL refuses two ranks on one device)
    // and only without a halo: the middle third is not checked to read owned columns only, and it
    // runs unordered with the exchange that fills the halo rows
    const char *force_env = getenv("MSPMV_DIST_FORCE_SPLIT");
    const bool force = force_env && atoi(force_env) != 0 && d->n_own >= 3 && n_halo == 0;
    if ((nranks > 1 && n_halo > 0) || force) {
        const int *ro = local_rows->row_offsets;
        int best_lo = 0, best_hi = 0, cur = 0;
        for (int r = 0; r <= d->n_own; ++r) {
            bool inner = r < d->n_own;
            for (int k = inner ? ro[r] : 0; inner && k < ro[r + 1]; ++k)
                inner = lcols[k] < d->n_own;
            if (!inner) {
                if (r - cur > best_hi - best_lo) {
                    best_lo = cur;
                    best_hi = r;
                }
                cur = r + 1;
            }
        }
        if (force) {
            best_lo = d->n_own / 3;
            best_hi = 2 * (d->n_own / 3);
        }
        if (force || 2LL * (ro[best_hi] - ro[best_lo]) >= (long long)nnz) {
            d->int_lo = best_lo;
            d->int_hi = best_hi;
            // the parts are row-range views of the local handle: their own row offsets, streams and
            // plans, the local handle's columns and values (no second copy of the matrix)
            const int cut[4] = {0, best_lo, best_hi, d->n_own};
            for (int q = 0; q < 3; ++q)
                if ((st = csr_create_view(d->local, cut[q], cut[q + 1], ro, &d->part[q])) != MSPMV_OK)
                    return bail(st);
            for (auto &e : d->ev)
                if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                    return bail(fail_msg(MSPMV_ERR_HIP, "dist_create: hipEventCreate"));
        }
    }
    hipStream_t s = d->local->stream;
    // request lists: every rank learns the counts matrix, then sends each owner the global
    // ids it needs; the owner keeps them (as local rows) as its send list to that rank
    int *d_cnt = nullptr, *d_cnt_all = nullptr, *d_halo = nullptr, *d_req = nullptr;
    auto cleanup = [&]() {
        dfree(d_cnt);
        dfree(d_cnt_all);
        dfree(d_halo);
        dfree(d_req);
    };
    if ((st = dalloc(&d_cnt, nranks)) != MSPMV_OK || (st = dalloc(&d_cnt_all, (size_t)nranks * nranks)) != MSPMV_OK ||
        (st = dalloc(&d_halo, halo.size())) != MSPMV_OK) {
        cleanup();
        return bail(st);
    }
    std::vector<int> cnt_all((size_t)nranks * nranks);
    hipError_t he = hipMemcpy(d_cnt, halo_counts.data(), sizeof(int) * nranks, hipMemcpyHostToDevice);
    if (he == hipSuccess && n_halo)
        he = hipMemcpy(d_halo, halo.data(), sizeof(int) * n_halo, hipMemcpyHostToDevice);
    if (he != hipSuccess) {
        cleanup();
        return bail(fail_msg(MSPMV_ERR_HIP, "dist_create: upload"));
    }
    nr = ncclAllGather(d_cnt, d_cnt_all, nranks, ncclInt32, d->comm, s);
    if (nr == ncclSuccess && hipStreamSynchronize(s) == hipSuccess &&
        hipMemcpy(cnt_all.data(), d_cnt_all, sizeof(int) * nranks * nranks, hipMemcpyDeviceToHost) == hipSuccess) {
    } else {
        cleanup();
        return bail(fail_msg(MSPMV_ERR_RCCL, "dist_create: count all-gather failed"));
    }
    d->send_counts.assign(nranks, 0);
    d->send_displs.assign(nranks + 1, 0);
    d->recv_counts.assign(halo_counts.begin(), halo_counts.end());
    d->recv_displs.assign(nranks + 1, 0);
    for (int g = 0; g < nranks; ++g) {
        d->send_counts[g] = cnt_all[(size_t)g * nranks + rank];  // rows rank g needs from me
        d->send_displs[g + 1] = d->send_displs[g] + d->send_counts[g];
        d->recv_displs[g + 1] = d->recv_displs[g] + d->recv_counts[g];
    }
    d->n_send = d->send_displs[nranks];
    if ((st = dalloc(&d_req, d->n_send)) != MSPMV_OK) {
        cleanup();
        return bail(st);
    }
    nr = ncclGroupStart();
    for (int g = 0; g < nranks && nr == ncclSuccess; ++g) {
        if (g == rank)
            continue;
        if (d->recv_counts[g])
            nr = ncclSend(d_halo + d->recv_displs[g], d->recv_counts[g], ncclInt32, g, d->comm, s);
        if (nr == ncclSuccess && d->send_counts[g])
            nr = ncclRecv(d_req + d->send_displs[g], d->send_counts[g], ncclInt32, g, d->comm, s);
    }
    ncclResult_t nr2 = ncclGroupEnd();
    if (nr != ncclSuccess || nr2 != ncclSuccess || hipStreamSynchronize(s) != hipSuccess) {
        cleanup();
        return bail(fail_msg(MSPMV_ERR_RCCL, "dist_create: request exchange failed"));
    }
    std::vector<int> req((size_t)std::max(d->n_send, 1));
    if (d->n_send && hipMemcpy(req.data(), d_req, sizeof(int) * d->n_send, hipMemcpyDeviceToHost) != hipSuccess) {
        cleanup();
        return bail(fail_msg(MSPMV_ERR_HIP, "dist_create: request download"));
    }
    cleanup();
    for (int k = 0; k < d->n_send; ++k) {
        req[k] -= lo;
        if (req[k] < 0 || req[k] >= d->n_own)
            return bail(fail_msg(MSPMV_ERR_INVALID, "dist_create: a peer requested a row this rank does not own"));
    }
    if ((st = dalloc(&d->d_send_idx, d->n_send)) != MSPMV_OK)
        return bail(st);
    if (d->n_send &&
        hipMemcpy(d->d_send_idx, req.data(), sizeof(int) * d->n_send, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail_msg(MSPMV_ERR_HIP, "dist_create: send list upload"));
    if ((st = dalloc(&d->d_ctrl, 1)) != MSPMV_OK)
        return bail(st);
    if (hipHostMalloc((void **)&d->h_ctrl, sizeof(CgControl) * 2, hipHostMallocDefault) != hipSuccess)
        return bail(fail_msg(MSPMV_ERR_HIP, "hipHostMalloc failed"));
    *out = d;
    return MSPMV_OK;
}

mspmv_status mspmv_dist_info(mspmv_dist d, int *n_own, int *n_halo, int *n_send)
{
    if (!d)
        return fail_msg(MSPMV_ERR_INVALID, "null dist");
    if (n_own)
        *n_own = d->n_own;
    if (n_halo)
        *n_halo = d->n_halo;
    if (n_send)
        *n_send = d->n_send;
    return MSPMV_OK;
}

}  // extern "C"

namespace {

mspmv_status ensure_buffers(mspmv_dist_s *d, int L, int nblk, int num_tiles, int hist_cap)
{
    if (L > d->cap_L) {
        dfree(d->d_pext);
        dfree(d->d_send);
        dfree(d->d_r);
        dfree(d->d_ap);
        dfree(d->d_scal);
        dfree(d->d_conv);
        dfree(d->d_red);
        d->cap_L = 0;
        D_ST(dalloc(&d->d_pext, (size_t)(d->n_own + d->n_halo) * L));
        D_ST(dalloc(&d->d_send, (size_t)d->n_send * L));
        D_ST(dalloc(&d->d_r, (size_t)d->n_own * L));
        D_ST(dalloc(&d->d_ap, (size_t)d->n_own * L));
        D_ST(dalloc(&d->d_scal, (size_t)L));
        D_ST(dalloc(&d->d_conv, (size_t)L));
        D_ST(dalloc(&d->d_red, (size_t)2 * L));
        d->cap_L = L;
    }
    const size_t slots = (size_t)std::max(nblk, num_tiles);
    const size_t pc = partials_capacity(slots, L);
    if (pc > d->partials_cap) {
        dfree(d->d_partials);
        d->partials_cap = 0;
        D_ST(dalloc(&d->d_partials, pc));
        d->partials_cap = pc;
    }
    if (gtickets_capacity(slots) > d->gtickets_cap) {
        dfree(d->d_gtickets);
        d->gtickets_cap = 0;
        D_ST(dalloc(&d->d_gtickets, gtickets_capacity(slots)));
        // on the local stream (non-blocking: a null-stream memset is not ordered before the folds on it)
        D_HIP(hipMemsetAsync(d->d_gtickets, 0, sizeof(unsigned) * gtickets_capacity(slots), d->local->stream));
        d->gtickets_cap = gtickets_capacity(slots);
    }
    if (hist_cap > d->hist_cap) {
        dfree(d->d_hist);
        d->hist_cap = 0;
        D_ST(dalloc(&d->d_hist, (size_t)hist_cap));
        d->hist_cap = hist_cap;
    }
    return MSPMV_OK;
}

// Pack the owned rows peers need and exchange them into the halo rows of d_pext.
mspmv_status halo_exchange(mspmv_dist_s *d, int L, const CgControl *ctrl)
{
    hipStream_t s = d->local->stream;
    D_HIP(launch_dist_pack(d->d_pext, d->d_send_idx, (long long)d->n_send * L, L, d->d_send, ctrl, s));
    if (d->nranks == 1)
        return MSPMV_OK;
    D_NCCL(ncclGroupStart());
    for (int g = 0; g < d->nranks; ++g) {
        if (g == d->rank)
            continue;
        if (d->send_counts[g])
            D_NCCL(ncclSend(d->d_send + (size_t)d->send_displs[g] * L, (size_t)d->send_counts[g] * L, ncclFloat64, g,
                            d->comm, s));
        if (d->recv_counts[g])
            D_NCCL(ncclRecv(d->d_pext + (size_t)(d->n_own + d->recv_displs[g]) * L, (size_t)d->recv_counts[g] * L,
                            ncclFloat64, g, d->comm, s));
    }
    D_NCCL(ncclGroupEnd());
    return MSPMV_OK;
}

mspmv_status get_local_plan(mspmv_dist_s *d, int L, const TilePlan **plan)
{
    // the plan the local handle's kernels use for L (the node-block plan for L > 1 on FEM blocks)
    return plan_for(d->local, L, plan);
}

}  // namespace

extern "C" {

mspmv_status mspmv_dist_x_ext(mspmv_dist d, int L, double **d_x_ext)
{
    if (!d || !d_x_ext || L < 1)
        return fail_msg(MSPMV_ERR_INVALID, "dist_x_ext: bad arguments");
    D_HIP(hipSetDevice(d->device));
    D_ST(ensure_buffers(d, L, 1, 1, 0));
    *d_x_ext = d->d_pext;
    return MSPMV_OK;
}

mspmv_status mspmv_dist_sync(mspmv_dist d)
{
    if (!d)
        return fail_msg(MSPMV_ERR_INVALID, "null dist");
    D_HIP(hipSetDevice(d->device));
    D_HIP(hipStreamSynchronize(d->local->stream));
    return MSPMV_OK;
}

mspmv_status mspmv_dist_time_local_dev(mspmv_dist d, double *d_Y_own, int L, int reps, double *avg_ms)
{
    if (!d || !avg_ms || L < 1 || reps < 1)
        return fail_msg(MSPMV_ERR_INVALID, "dist_time_local: bad arguments");
    D_HIP(hipSetDevice(d->device));
    D_ST(ensure_buffers(d, L, 1, 1, 0));
    // the row ranges the overlapped SpMM launches (or the whole local matrix), back to back on
    // one stream, events around the region only (per-launch events would inflate it)
    mspmv_handle hs[3];
    const double *xs[3];
    double *ys[3];
    int n = 0;
    const int offs[3] = {0, d->int_lo, d->int_hi};
    if (!d->part[1]) {
        hs[0] = d->local;
        xs[0] = d->d_pext;
        ys[0] = d_Y_own;
        n = 1;
    }
    for (int q = 0; q < 3 && d->part[1]; ++q)
        if (d->part[q]->m > 0) {
            hs[n] = d->part[q];
            xs[n] = d->d_pext;
            ys[n] = d_Y_own + (size_t)offs[q] * L;
            ++n;
        }
    double kern = 0.0;
    int kps = 0;
    return mspmv_time_spmm_batch_dev(n, hs, xs, ys, L, reps, avg_ms, &kern, &kps);
}

mspmv_status mspmv_dist_spmm_dev(mspmv_dist d, const double *d_X_own, double *d_Y_own, int L)
{
    if (!d)
        return fail_msg(MSPMV_ERR_INVALID, "null dist");
    if (L < 1)
        return fail_msg(MSPMV_ERR_INVALID, "L must be >= 1");
    D_HIP(hipSetDevice(d->device));
    D_ST(ensure_buffers(d, L, 1, 1, 0));
    hipStream_t s = d->local->stream;
    if (d->n_own && d_X_own != d->d_pext)
        D_HIP(hipMemcpyAsync(d->d_pext, d_X_own, sizeof(double) * (size_t)d->n_own * L, hipMemcpyDeviceToDevice, s));
    if (!d->part[1]) {  // no interior split: exchange, then the whole local SpMM
        D_ST(halo_exchange(d, L, nullptr));
        return mspmv_dspmm_dev(d->local, d->d_pext, d_Y_own, L);
    }
    // interior rows on their own stream while this stream packs and exchanges the halo
    mspmv_handle head = d->part[0], mid = d->part[1], tail = d->part[2];
    D_HIP(hipEventRecord(d->ev[0], s));
    D_HIP(hipStreamWaitEvent(mid->stream, d->ev[0], 0));
    D_ST(mspmv_dspmm_dev(mid, d->d_pext, d_Y_own + (size_t)d->int_lo * L, L));
    D_HIP(hipEventRecord(d->ev[1], mid->stream));
    D_ST(halo_exchange(d, L, nullptr));
    D_HIP(hipEventRecord(d->ev[2], s));
    const int offs[2] = {0, d->int_hi};
    mspmv_handle ends[2] = {head, tail};
    for (int q = 0; q < 2; ++q) {
        if (ends[q]->m == 0)
            continue;
        D_HIP(hipStreamWaitEvent(ends[q]->stream, d->ev[2], 0));
        D_ST(mspmv_dspmm_dev(ends[q], d->d_pext, d_Y_own + (size_t)offs[q] * L, L));
        D_HIP(hipEventRecord(d->ev[3 + q], ends[q]->stream));
        D_HIP(hipStreamWaitEvent(s, d->ev[3 + q], 0));
    }
    D_HIP(hipStreamWaitEvent(s, d->ev[1], 0));
    return MSPMV_OK;
}

static mspmv_status dist_cg_native(mspmv_dist d, const double *d_B_own, double *d_X_own, int L, int max_iters,
                                   double tolerance, int *iters, double *max_err_hist, int hist_cap);

// Any L: the L recurrences are independent per column (no_pretreatment.hpp:109-120,163-176), so a
// width outside {1, 2, 4, 8, 16} is solved as column groups of native widths, one after another,
// each a collective solve that every rank runs in the same order; iteration count = the groups'
// maximum, history = the max over groups with finished groups frozen (mspmv_dcg_multi's rule).
mspmv_status mspmv_dist_cg_dev(mspmv_dist d, const double *d_B_own, double *d_X_own, int L, int max_iters,
                               double tolerance, int *iters, double *max_err_hist, int hist_cap)
{
    if (!d)
        return fail_msg(MSPMV_ERR_INVALID, "null dist");
    if (L < 1)
        return fail_msg(MSPMV_ERR_INVALID, "L must be >= 1");
    if (supported_L(L))
        return dist_cg_native(d, d_B_own, d_X_own, L, max_iters, tolerance, iters, max_err_hist, hist_cap);
    D_HIP(hipSetDevice(d->device));
    const size_t m = (size_t)std::max(d->n_own, 1);
    const int cap = max_err_hist ? std::max(hist_cap, 0) : 0;
    double *gb = nullptr, *gx = nullptr;
    D_ST(dalloc(&gb, m * 16));
    mspmv_status st = dalloc(&gx, m * 16);
    hipStream_t s = d->local->stream;
    std::vector<std::vector<double>> gh;
    std::vector<int> git;
    int total = 0;
    bool broke = false, faulted = false;
    for (int c0 = 0; c0 < L && st == MSPMV_OK;) {
        int w = 16;
        while (w > L - c0)
            w >>= 1;
        if (d->n_own && launch_panel_copy(d_B_own + c0, L, gb, w, (long long)d->n_own, w, w, s) != hipSuccess) {
            st = fail_msg(MSPMV_ERR_HIP, "dist CG: column group copy");
            break;
        }
        std::vector<double> hg((size_t)std::max(cap, 1));
        int it = 0;
        st = dist_cg_native(d, gb, gx, w, max_iters, tolerance, &it, cap ? hg.data() : nullptr, cap);
        if (st == MSPMV_ERR_BREAKDOWN) {
            broke = true;
            st = MSPMV_OK;
        } else if (st == MSPMV_ERR_FAULT) {  // the other groups still run (each solve re-zeroes its tickets)
            faulted = true;
            st = MSPMV_OK;
        }
        if (st == MSPMV_OK && d->n_own &&
            (launch_panel_copy(gx, w, d_X_own + c0, L, (long long)d->n_own, w, w, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess))
            st = fail_msg(MSPMV_ERR_HIP, "dist CG: column group copy back");
        total = std::max(total, it);
        gh.push_back(std::move(hg));
        git.push_back(it);
        c0 += w;
    }
    dfree(gb);
    dfree(gx);
    if (iters)
        *iters = total;
    for (int k = 0; k < std::min(total, cap); ++k) {
        double v = 0.0;
        for (size_t g = 0; g < gh.size(); ++g)
            if (git[g] > 0)
                v = std::max(v, gh[g][(size_t)std::min(k, git[g] - 1)]);
        max_err_hist[k] = v;
    }
    if (st == MSPMV_OK && faulted)
        return fail_msg(MSPMV_ERR_FAULT, "dist CG: a reduction ticket drew past its group in at least one column "
                                         "group: X is not a solution");
    if (st == MSPMV_OK && broke)
        return fail_msg(MSPMV_ERR_BREAKDOWN, "dist CG breakdown: non-finite alpha in at least one column (frozen)");
    return st;
}

static mspmv_status dist_cg_native(mspmv_dist d, const double *d_B_own, double *d_X_own, int L, int max_iters,
                                   double tolerance, int *iters, double *max_err_hist, int hist_cap)
{
    if (max_iters < 0)
        return fail_msg(MSPMV_ERR_INVALID, "max_iters < 0");
    D_HIP(hipSetDevice(d->device));
    const TilePlan *plan = nullptr;
    D_ST(get_local_plan(d, L, &plan));
    const long long elems = (long long)d->n_own * L;
    const int nblk = cg_update_blocks(std::max(elems, 2LL), d->local->num_cus);
    const int cap = max_err_hist ? std::max(hist_cap, 0) : 0;
    // overlapped iteration (the local rows split head | interior | tail, as mspmv_dist_spmm_dev):
    // each part's dot-mode tiles write their p.Ap partials at the part's offset, one fold sums
    // the three in tile order
    const TilePlan *pp[3] = {nullptr, nullptr, nullptr};
    // offset windows (mspmv_dia.hip) where the rows take them -- the unsplit local rows, or a part whose
    // columns keep a constant offset from its rows (the interior: owned columns only); their dot mode
    // writes one p.Ap partial per window into the same fold (MSPMV_DIA_DOT=0: tiles everywhere)
    const TilePlan *dlocal = nullptr, *dpart[3] = {nullptr, nullptr, nullptr};
    int toff[4] = {0, 0, 0, 0};
    const bool split = d->part[1] != nullptr;
    if (dia_dot_fused() && !split)
        D_ST(dia_plan_for(d->local, L, &dlocal));
    for (int q = 0; q < 3 && split; ++q) {
        D_ST(plan_for(d->part[q], L, &pp[q]));
        if (dia_dot_fused())
            D_ST(dia_plan_for(d->part[q], L, &dpart[q]));
        toff[q + 1] = toff[q] + (dpart[q] ? dpart[q]->num_tiles : pp[q]->num_tiles);
    }
    D_ST(ensure_buffers(d, L, nblk, std::max({plan->num_tiles, dlocal ? dlocal->num_tiles : 0, toff[3]}), cap));
    hipStream_t s = d->local->stream;
    DistVecArgs va{};
    va.n_elems = elems;
    va.x = d_X_own;
    va.r = d->d_r;
    va.p = d->d_pext;
    va.p0 = d->d_pext;
    va.ap = d->d_ap;
    va.scal = d->d_scal;
    va.ctrl = d->d_ctrl;
    va.conv = d->d_conv;
    va.partials = d->d_partials;
    va.gtickets = d->d_gtickets;
    va.hist = cap ? d->d_hist : nullptr;
    va.hist_cap = cap;
    va.tol = tolerance;
    double *pAp = d->d_red, *rr = d->d_red + L;
    // init: x = 0, r = p = b; all-reduce b.b; scalars
    D_HIP(hipMemsetAsync(d->d_ctrl, 0, sizeof(CgControl), s));
    // a ticket fault does not stop the device side of a sharded solve: every rank must stop at the same
    // batch, so the host stops on the all-reduced fault word (below)
    D_HIP(hipMemsetD32Async((hipDeviceptr_t)&d->d_ctrl->fault_no_stop, 1, 1, s));
    // split-row tickets reset themselves when every tile sharing a row closes it; a CG SpMM that returns
    // at its stop test leaves them as they were, so every solve starts from zeroed ones
    for (const TilePlan *tp : {plan, pp[0], pp[1], pp[2], dlocal, dpart[0], dpart[1], dpart[2]})
        if (tp && tp->d_fix_cnt)
            D_HIP(hipMemsetAsync(tp->d_fix_cnt, 0, sizeof(unsigned) * (size_t)tp->num_tiles, s));
    // test hook: fold tickets dirty at the first fold (round 5's unordered zeroing of recycled memory)
    const int poison = d->poison_flags;
    d->poison_flags = 0;
    // fold tickets: zeroed at every solve's start (a solve that stopped early or faulted may leave some raised)
    D_HIP(hipMemsetAsync(d->d_gtickets, 0, sizeof(unsigned) * d->gtickets_cap, s));
    {
        DistVecArgs a = va;
        a.p = d_B_own;
        a.red_out = rr;
        D_HIP(launch_dist_vec_mirror(0, a, L, nblk, nullptr, s));
        D_NCCL(ncclAllReduce(rr, rr, L, ncclFloat64, ncclSum, d->comm, s));
        a.red_in = rr;
        D_HIP(launch_dist_vec_mirror(1, a, L, 1, nullptr, s));
    }
    if (poison & MSPMV_POISON_FILL)  // test hook: the iterations' folds meet dirty tickets (after the init's)
        D_HIP(hipMemsetD32Async((hipDeviceptr_t)d->d_gtickets, (int)d->poison_value, d->gtickets_cap, s));
    auto iteration = [&]() -> mspmv_status {
        DistVecArgs a = va;
        D_HIP(launch_dist_vec_mirror(2, a, L, nblk, d->d_pext, s));       // p = r + beta p
        if (!split) {
            D_ST(halo_exchange(d, L, d->d_ctrl));                           // p halo rows
            if (dlocal) {
                D_HIP(launch_dia(d->local, *dlocal, d->d_pext, d->d_ap, L, L, d->d_ctrl, d->d_partials));
                D_HIP(launch_fold_dot(dlocal->num_tiles, L, d->d_partials, d->d_gtickets, pAp, nullptr, nullptr,
                                      d->d_ctrl, -1, s));
            } else {
                D_HIP(launch_spmm_dot(d->local, *plan, d->d_pext, d->d_ap, L, d->d_ctrl, d->d_partials, d->d_gtickets,
                                      pAp));
            }
        } else {
            const int rofs[3] = {0, d->int_lo, d->int_hi};
            auto part_dot = [&](int q, hipStream_t st) -> hipError_t {
                double *ap = d->d_ap + (size_t)rofs[q] * L, *part = d->d_partials + (size_t)toff[q] * L;
                return dpart[q] ? launch_dia(d->part[q], *dpart[q], d->d_pext, ap, L, L, d->d_ctrl, part, rofs[q], st)
                                : launch_spmm_dot_tiles(d->part[q], *pp[q], d->d_pext, ap, L, d->d_ctrl, part, st,
                                                        rofs[q]);
            };
            // the interior (owned columns only) on its own stream beside the exchange
            mspmv_handle mid = d->part[1];
            D_HIP(hipEventRecord(d->ev[0], s));
            D_HIP(hipStreamWaitEvent(mid->stream, d->ev[0], 0));
            D_HIP(part_dot(1, mid->stream));
            D_HIP(hipEventRecord(d->ev[1], mid->stream));
            D_ST(halo_exchange(d, L, d->d_ctrl));                           // p halo rows
            for (int q = 0; q < 3; q += 2)
                D_HIP(part_dot(q, s));
            D_HIP(hipStreamWaitEvent(s, d->ev[1], 0));
            D_HIP(launch_fold_dot(toff[3], L, d->d_partials, d->d_gtickets, pAp, nullptr, nullptr, d->d_ctrl, -1, s));
        }
        D_NCCL(ncclAllReduce(pAp, pAp, L, ncclFloat64, ncclSum, d->comm, s));
        a.red_in = pAp;
        a.red_out = rr;
        D_HIP(launch_dist_vec_mirror(3, a, L, nblk, nullptr, s));          // x, r, local r.r
        D_NCCL(ncclAllReduce(rr, rr, L, ncclFloat64, ncclSum, d->comm, s));
        D_HIP(launch_dist_vec_mirror(4, a, L, 1, nullptr, s));             // stop test, beta
        return MSPMV_OK;
    };
    int iterations_enqueued = 0;
    auto iteration_hook = [&]() -> mspmv_status {
        D_ST(iteration());
        if ((poison & MSPMV_POISON_LATE_ZERO) && ++iterations_enqueued == 1)  // the late zeroing
            D_HIP(hipMemsetAsync(d->d_gtickets, 0, sizeof(unsigned) * d->gtickets_cap, s));
        return MSPMV_OK;
    };
    // batches of K iterations, the control word of batch b inspected while b+1 is queued
    const int K = cg_batch_iters(d->n_own, d->local->nnz, L);
    // MSPMV_DIST_GRAPH: 1 on, 0 off; unset: on for a single rank (tested bit-identical to eager),
    // off for several ranks -- RCCL collectives replayed from a captured graph have only run at
    // world 1 here (RCCL refuses two ranks on one device), so the driver's multi-GPU runs keep the
    // eager enqueue unless asked
    static const int graph_env = [] {
        const char *e = getenv("MSPMV_DIST_GRAPH");
        return e ? (atoi(e) != 0 ? 1 : 0) : -1;
    }();
    const bool use_graph = (graph_env >= 0 ? graph_env == 1 : d->nranks == 1) && !(poison & MSPMV_POISON_LATE_ZERO);
    const void *tk = nullptr;
    static_assert(sizeof(tk) == sizeof(tolerance), "tolerance bits as a key word");
    std::memcpy(&tk, &tolerance, sizeof tk);
    const std::vector<const void *> key = {
        d_X_own, d->d_pext, d->d_send, d->d_r, d->d_ap, d->d_partials, d->d_gtickets, d->d_scal, d->d_conv,
        d->d_red, d->d_ctrl, va.hist, plan, pp[0], pp[1], pp[2], dlocal, dpart[0], dpart[1], dpart[2], tk,
        reinterpret_cast<const void *>((intptr_t)L),
        reinterpret_cast<const void *>((intptr_t)nblk), reinterpret_cast<const void *>((intptr_t)cap),
        reinterpret_cast<const void *>((intptr_t)K)};
    // one batch: the cached graph when it matches (capturing it now if this object has run an eager
    // batch before), else the iterations enqueued one by one
    auto batch = [&](int k) -> mspmv_status {
        if (use_graph && k == K && d->cg_warm && (!d->cg_exec || d->cg_key != key)) {
            if (d->cg_exec)
                (void)hipGraphExecDestroy(d->cg_exec);
            if (d->cg_graph)
                (void)hipGraphDestroy(d->cg_graph);
            d->cg_exec = nullptr;
            d->cg_graph = nullptr;
            d->cg_key.clear();
            hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
            mspmv_status cst = e == hipSuccess ? MSPMV_OK : MSPMV_ERR_HIP;
            for (int i = 0; i < K && cst == MSPMV_OK; ++i)
                cst = iteration();
            hipGraph_t g = nullptr;
            const hipError_t e2 = e == hipSuccess ? hipStreamEndCapture(s, &g) : e;
            d->cg_graph = g;
            if (cst == MSPMV_OK && e2 == hipSuccess &&
                hipGraphInstantiate(&d->cg_exec, g, nullptr, nullptr, 0) == hipSuccess) {
                d->cg_key = key;
                if (getenv("MSPMV_DEBUG_GRAPH"))
                    fprintf(stderr, "mspmv: dist CG batch of %d iterations captured (rank %d)\n", K, d->rank);
            } else {
                fprintf(stderr, "mspmv: dist CG batch capture failed (rank %d): batches run eagerly\n", d->rank);
                // capture unsupported here (or failed): this object runs its batches eagerly from now on
                if (d->cg_graph)
                    (void)hipGraphDestroy(d->cg_graph);
                d->cg_graph = nullptr;
                d->cg_exec = nullptr;
                d->cg_warm = false;
                (void)hipGetLastError();
                // whatever failed inside the capture (HIP or RCCL), this batch still runs eagerly
                // below: the other ranks enqueue theirs, so skipping it would misalign the
                // collectives across ranks (a hang, not an error)
                (void)cst;
            }
        }
        if (use_graph && k == K && d->cg_exec && d->cg_key == key)
            return hipGraphLaunch(d->cg_exec, s) == hipSuccess ? MSPMV_OK
                                                               : fail_msg(MSPMV_ERR_HIP, "dist CG: graph launch failed");
        for (int i = 0; i < k; ++i)
            D_ST(iteration_hook());
        return MSPMV_OK;
    };
    hipEvent_t evs[2] = {nullptr, nullptr};
    D_HIP(hipEventCreateWithFlags(&evs[0], hipEventDisableTiming));
    D_HIP(hipEventCreateWithFlags(&evs[1], hipEventDisableTiming));
    mspmv_status st = MSPMV_OK;
    int launched = 0, pending = 0, oldest = 0, slot = 0;
    while (st == MSPMV_OK) {
        const int k = std::min(K, max_iters - launched);
        if (k > 0) {
            st = batch(k);
            if (st != MSPMV_OK)
                break;
            // every rank's fault word -> the max over ranks, so all ranks stop at the same batch
            if (d->nranks > 1 &&
                ncclAllReduce(&d->d_ctrl->fault, &d->d_ctrl->fault, 1, ncclUint32, ncclMax, d->comm, s) != ncclSuccess) {
                st = fail_msg(MSPMV_ERR_RCCL, "dist CG: fault word all-reduce failed");
                break;
            }
            if (hipMemcpyAsync(&d->h_ctrl[slot], d->d_ctrl, sizeof(CgControl), hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipEventRecord(evs[slot], s) != hipSuccess) {
                st = fail_msg(MSPMV_ERR_HIP, "dist CG: control copy failed");
                break;
            }
            launched += k;
            ++pending;
            slot ^= 1;
        }
        if (pending == 0)
            break;
        if (pending == 2 || k <= 0) {
            if (hipEventSynchronize(evs[oldest]) != hipSuccess) {
                st = fail_msg(MSPMV_ERR_HIP, "dist CG: event sync failed");
                break;
            }
            --pending;
            d->cg_warm = true;  // a batch has run: RCCL's connections exist, later batches may be captured
            const bool done = d->h_ctrl[oldest].done != 0 ||
                              (d->h_ctrl[oldest].fault != 0 && !(poison & MSPMV_POISON_NO_STOP));
            oldest ^= 1;
            if (done)
                break;
        }
    }
    // every rank reaches the same decision (the control word is a function of all-reduced
    // values), so all ranks have enqueued the same collectives
    hipError_t e = hipStreamSynchronize(s);
    CgControl fin{};
    if (e == hipSuccess)
        e = hipMemcpy(&fin, d->d_ctrl, sizeof(CgControl), hipMemcpyDeviceToHost);
    (void)hipEventDestroy(evs[0]);
    (void)hipEventDestroy(evs[1]);
    if (st != MSPMV_OK)
        return st;
    if (e != hipSuccess)
        return fail_msg(MSPMV_ERR_HIP, std::string("dist CG finish: ") + hipGetErrorString(e));
    const int it = fin.done ? fin.iters_out : fin.iter;
    if (iters)
        *iters = it;
    if (cap > 0) {
        const int nh = std::min(it, cap);
        if (nh > 0)
            D_HIP(hipMemcpy(max_err_hist, d->d_hist, sizeof(double) * nh, hipMemcpyDeviceToHost));
    }
    if (fin.fault)
        return fail_msg(MSPMV_ERR_FAULT, "dist CG: a reduction ticket drew past its group (the ticket array was not "
                                         "zero when a fold began): X is not a solution");
    if (fin.breakdown)
        return fail_msg(MSPMV_ERR_BREAKDOWN, "dist CG breakdown: non-finite alpha at iteration " + std::to_string(it));
    return MSPMV_OK;
}

mspmv_status mspmv_dist_test_poison_tickets(mspmv_dist d, unsigned value, int flags)
{
    if (!d)
        return fail_msg(MSPMV_ERR_INVALID, "null dist");
    if (flags & ~(MSPMV_POISON_FILL | MSPMV_POISON_LATE_ZERO | MSPMV_POISON_NO_STOP))
        return fail_msg(MSPMV_ERR_INVALID, "dist_test_poison_tickets: unknown flag");
    d->poison_value = value;
    d->poison_flags = flags;
    return MSPMV_OK;
}

}  // extern "C"
