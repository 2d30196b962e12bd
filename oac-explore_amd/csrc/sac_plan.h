// The plan object behind an oac_sac handle (SAC twin-critic and particle
// K-head trainers share it; each kind has its own workspace layout and
// launch sequence).
#pragma once
#include "../../include/oac_amd.h"
#include "plan_common.h"

namespace oac {

constexpr int kMaxWs = 128;

struct SacPlan : PlanBase {
  oac_sac_config c;
  oac_sac_layout L;
  oac_sac_buffers b;
  WsBuf ws[kMaxWs];
  Split sp_q0, sp_q1, sp_ql, sp_p0, sp_p1, sp_ph;

  float* W(int id) const { return b.workspace + ws[id].off; }
  float* P(int64_t off) const { return b.params + off; }
  float* T(int64_t off) const { return b.targets + off; }
  StepState* state() const { return reinterpret_cast<StepState*>(b.step_state); }
  AlphaState* alpha() const { return reinterpret_cast<AlphaState*>(b.alpha_state); }
};


// particle trainer (particle_plan.hip)
void particle_layout_workspace(SacPlan& p);
int particle_run_step(SacPlan& p, int flags, hipStream_t s);
int particle_step_phase(SacPlan& p, int phase, int flags, hipStream_t s);
void particle_plan_splits(SacPlan& p);

}  // namespace oac
