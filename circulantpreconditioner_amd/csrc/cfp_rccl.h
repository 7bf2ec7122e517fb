// RCCL communicators of the library: non-blocking creation against a deadline, the poll every
// call on a non-blocking communicator needs, and what RCCL the process actually bound.
//
// A communicator made with ncclConfig_t.blocking = 0 returns from ncclCommInitRankConfig at
// once and reports ncclInProgress until every rank has joined; the same holds for
// ncclGroupEnd / ncclAllReduce / ncclCommFinalize on it.  The documented protocol is to poll
// ncclCommGetAsyncError until the state leaves ncclInProgress.  Polling with a deadline turns a
// peer that never arrives (the first real 8-rank run of a driver, a wrong unique id) into an
// error the caller can report, where the blocking ncclCommInitRank would hang the process.
#pragma once

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace cfp {

constexpr double kRcclDefaultTimeoutS = 300.0;

// CFP_RCCL_BLOCKING=1 in the environment selects the blocking protocol instead: ncclCommInitRank
// (no deadline: a missing peer hangs, as with any plain RCCL program) and ncclCommDestroy, with
// every call returning only when it is done.  It is the known-good fallback for a first run
// between real peers, where the non-blocking group end and the polled finalize have not run
// before.  Read once per process, so creation and destruction agree.
inline bool rccl_blocking() {
  static const bool b = [] {
    const char* e = std::getenv("CFP_RCCL_BLOCKING");
    return e && *e && std::strcmp(e, "0") != 0;
  }();
  return b;
}

// Wait until `c` leaves ncclInProgress; `r` is the result of the call just made on it.  A
// blocking communicator never reports ncclInProgress, so this is a no-op there.  Returns the
// final state, or ncclInProgress if `deadline_s` (> 0) passed first.
inline ncclResult_t rccl_settle(ncclComm_t c, ncclResult_t r, double deadline_s) {
  if (r != ncclInProgress || !c) return r;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t q = ncclCommGetAsyncError(c, &st);
    if (q != ncclSuccess) return q;
    if (st != ncclInProgress) return st;
    if (deadline_s > 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > deadline_s)
      return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// ncclCommInitRankConfig with blocking = 0, polled against `timeout_s`.  On failure or timeout
// the half-made communicator is aborted, *comm is NULL and *timed_out says which.  Under
// CFP_RCCL_BLOCKING, ncclCommInitRank without a deadline.
inline ncclResult_t rccl_init_rank(ncclComm_t* comm, int nranks, const ncclUniqueId& id, int rank, double timeout_s,
                                   bool* timed_out) {
  *comm = nullptr;
  *timed_out = false;
  if (rccl_blocking()) {
    const ncclResult_t nr = ncclCommInitRank(comm, nranks, id, rank);
    if (nr != ncclSuccess) *comm = nullptr;
    return nr;
  }
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  *comm = nullptr;
  *timed_out = false;
  ncclResult_t nr = ncclCommInitRankConfig(comm, nranks, id, rank, &cfg);
  if ((nr == ncclSuccess || nr == ncclInProgress) && *comm)
    nr = rccl_settle(*comm, ncclInProgress, timeout_s);  // success may still be in progress
  if (nr == ncclInProgress) *timed_out = true;
  if (nr != ncclSuccess && *comm) {
    ncclCommAbort(*comm);
    *comm = nullptr;
  }
  return nr;
}

// Finalize (flush, polled) and destroy; a communicator that does not quiesce within the deadline
// is aborted instead.  A blocking communicator (CFP_RCCL_BLOCKING) is destroyed directly.
inline void rccl_destroy(ncclComm_t c, double timeout_s) {
  if (!c) return;
  if (rccl_blocking()) {
    ncclCommDestroy(c);
    return;
  }
  ncclResult_t r = ncclCommFinalize(c);
  if (r == ncclSuccess || r == ncclInProgress) r = rccl_settle(c, ncclInProgress, timeout_s);
  if (r == ncclSuccess)
    ncclCommDestroy(c);
  else
    ncclCommAbort(c);
}

// Path of the shared object that defines the ncclCommInitRankConfig this library calls (torch
// carries its own librccl with the same soname; whichever the process loaded first wins).
inline void rccl_library_path(char* buf, int len) {
  if (!buf || len <= 0) return;
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(&ncclCommInitRankConfig), &info) && info.dli_fname)
    std::snprintf(buf, (size_t)len, "%s", info.dli_fname);
  else
    std::snprintf(buf, (size_t)len, "unknown");
}

}  // namespace cfp
