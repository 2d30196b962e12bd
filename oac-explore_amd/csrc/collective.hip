// RCCL transport for the data-parallel step's exchanges (the
// "oac_allreduce_hook / RCCL comm passed in" entry point; 8e: three in-place
// SUM all-reduces per step over xGMI).
//
// The reference has no distributed path (one independent seed per GPU,
// /root/reference/main.py:575-578); the build's DP step needs three exchanges
// per step (trainer/trainer.py:139-210 order: the alpha sum before the TD
// target, the critic gradients before the critic Adam, the policy gradients
// before the policy Adam).  The library issues them itself between its own
// launches (sac_plan.hip, run_step_dp) through an oac_allreduce_fn; this file
// is the RCCL implementation of that hook.
//
// librccl is loaded at run time from the path the caller passes -- the
// librccl.so its process already uses (torch's), so one RCCL instance serves
// torch's process group and this communicator -- and only five symbols are
// resolved.  rccl.h supplies the types; nothing links against librccl.
#include <dlfcn.h>

#include <cstring>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../../include/oac_amd.h"
#include "oac_common.h"

namespace oac {

struct RcclApi {
  void* so = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

static int load_rccl(const char* path, RcclApi& a) {
  if (!path || !*path) { set_error("rccl: no library path"); return 1; }
  a.so = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!a.so) { set_error("rccl: dlopen(%s): %s", path, dlerror()); return 1; }
  auto sym = [&](const char* name) -> void* {
    void* f = dlsym(a.so, name);
    if (!f) set_error("rccl: %s not found in %s", name, path);
    return f;
  };
  a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(sym("ncclGetUniqueId"));
  a.comm_init_rank = reinterpret_cast<decltype(a.comm_init_rank)>(sym("ncclCommInitRank"));
  a.all_reduce = reinterpret_cast<decltype(a.all_reduce)>(sym("ncclAllReduce"));
  a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(sym("ncclCommDestroy"));
  a.error_string = reinterpret_cast<decltype(a.error_string)>(sym("ncclGetErrorString"));
  if (!a.get_unique_id || !a.comm_init_rank || !a.all_reduce || !a.comm_destroy || !a.error_string) {
    dlclose(a.so);
    a.so = nullptr;
    return 1;
  }
  return 0;
}

}  // namespace oac

using namespace oac;

struct oac_rccl {
  RcclApi api;
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
};

extern "C" {

int oac_rccl_unique_id(const char* librccl_path, void* id128) {
  if (!id128) { set_error("rccl: null id buffer"); return 1; }
  RcclApi a;
  if (load_rccl(librccl_path, a)) return 1;
  ncclUniqueId id;
  const ncclResult_t r = a.get_unique_id(&id);
  if (r != ncclSuccess) { set_error("ncclGetUniqueId: %s", a.error_string(r)); return 1; }
  static_assert(sizeof(id) == NCCL_UNIQUE_ID_BYTES, "unique id size");
  std::memcpy(id128, &id, sizeof(id));
  // (the library stays loaded: dlclose of an RCCL instance torch also holds is a no-op)
  return 0;
}

int oac_rccl_create(const char* librccl_path, const void* id128, int rank, int world,
                    oac_rccl** out) {
  if (!id128 || !out) { set_error("rccl: null id / out"); return 1; }
  if (world < 1 || rank < 0 || rank >= world) { set_error("rccl: rank %d of %d", rank, world); return 1; }
  oac_rccl* c = new oac_rccl();
  if (load_rccl(librccl_path, c->api)) { delete c; return 1; }
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  // collective across the ranks: every rank calls this with the same id
  const ncclResult_t r = c->api.comm_init_rank(&c->comm, world, id, rank);
  if (r != ncclSuccess) {
    set_error("ncclCommInitRank(rank %d of %d): %s", rank, world, c->api.error_string(r));
    delete c;
    return 1;
  }
  c->rank = rank;
  c->world = world;
  *out = c;
  return 0;
}

int oac_rccl_destroy(oac_rccl* c) {
  if (!c) return 0;
  int rc = 0;
  if (c->comm) {
    const ncclResult_t r = c->api.comm_destroy(c->comm);
    if (r != ncclSuccess) { set_error("ncclCommDestroy: %s", c->api.error_string(r)); rc = 1; }
  }
  delete c;
  return rc;
}

// an oac_allreduce_fn: in-place fp32 SUM over the communicator, on `stream`
int oac_rccl_allreduce(void* ctx, float* buf, int64_t n, void* stream) {
  oac_rccl* c = static_cast<oac_rccl*>(ctx);
  if (!c || !c->comm) { set_error("rccl: no communicator"); return 1; }
  if (n <= 0) return 0;
  const ncclResult_t r = c->api.all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, c->comm,
                                           reinterpret_cast<hipStream_t>(stream));
  if (r != ncclSuccess) { set_error("ncclAllReduce(%lld floats): %s", (long long)n, c->api.error_string(r)); return 1; }
  return 0;
}

}  // extern "C"
