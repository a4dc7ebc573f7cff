// lgx_host.h — host (CPU) backend of include/lgx.h, selected by lgx_create(device < 0).
// Internal to liblgx.so: lgx_env.hip's C ABI dispatches here for host envs. Every buffer
// pointer in lgx_buffers is host memory; the stream arguments are ignored.
#pragma once
#include <stdint.h>

#include "../../include/lgx.h"

namespace lgxh {

// decimation x physics substeps (when `physics`) + post-physics for every env, OpenMP over
// envs; episode statistics of the envs that reset are summed in env order (deterministic).
void step(const lgx_model* M, const lgx_task_params* P, const lgx_buffers* B, uint64_t seed, uint64_t step,
          bool physics);
// reset_idx for the masked envs (RNG stream 1, counter = call)
void reset(const lgx_task_params* P, const lgx_buffers* B, const uint8_t* mask, uint64_t seed, uint64_t call);
// lgx_episode_extras on host buffers
void episode_extras(const lgx_task_params* P, const lgx_buffers* B, float* means, float* level_mean,
                    uint8_t* time_outs, uint64_t* step_counter);
// lgx_command_curriculum on host buffers
void command_curriculum(const lgx_task_params* P, const lgx_buffers* B, uint64_t seed, uint64_t step,
                        const double* global_sum_count);
// the worker threads the host backend uses (OpenMP)
int threads();

}  // namespace lgxh
