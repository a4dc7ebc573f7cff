/* placeholder: replaced below */
#include "lgx_oracle.h"
void oracle_physics_substep(const lgx_model* M, const lgx_task_params* P, lgx_buffers* B, int env) { (void)M; (void)P; (void)B; (void)env; }
double oracle_energy(const lgx_model* M, const lgx_task_params* P, const lgx_buffers* B, int env) { (void)M; (void)P; (void)B; (void)env; return 0; }
