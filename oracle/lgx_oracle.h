/* lgx_oracle.h — CPU oracle entry points (TEST INFRASTRUCTURE ONLY; see lgx_oracle.c). */
#ifndef LGX_ORACLE_H
#define LGX_ORACLE_H
#include <stdint.h>
#include "../include/lgx.h"

#ifdef __cplusplus
extern "C" {
#endif

void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void oracle_compute_torques(const lgx_task_params* P, const lgx_buffers* B, int env);
void oracle_physics_substep(const lgx_model* M, const lgx_task_params* P, lgx_buffers* B, int env);
void oracle_post_physics(const lgx_task_params* P, lgx_buffers* B, uint64_t seed, uint64_t step);
void oracle_reset_envs(const lgx_task_params* P, lgx_buffers* B, const uint8_t* mask, uint64_t seed, uint64_t call,
                       int after_init);
void oracle_clip_actions(const lgx_task_params* P, lgx_buffers* B);
void oracle_step(const lgx_model* M, const lgx_task_params* P, lgx_buffers* B, uint64_t seed, uint64_t step);
/* physics diagnostics (tests): kinetic + potential energy, total momentum */
double oracle_energy(const lgx_model* M, const lgx_task_params* P, const lgx_buffers* B, int env);
/* constraint rows of env's latest physics substep */
int oracle_debug_rows(int env);
int64_t oracle_sizeof_params(void);
int64_t oracle_sizeof_model(void);
int64_t oracle_sizeof_buffers(void);

#ifdef __cplusplus
}
#endif
#endif
