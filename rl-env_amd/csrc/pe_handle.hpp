// pe_handle.hpp -- the handle behind the opaque pe_handle* of include/plantos_batch.h
// (shared by the translation units of libplantos_hip.so; not part of the ABI).
#pragma once
#include "../../include/plantos_batch.h"
#include "pe_device.hpp"

struct pe_handle {
  int device;
  int n;
  pe_config cfg;
  pe::Geo g;
  pe::Rules rl;
  pe::State st;
  void* mem;
  size_t bytes;
  int variant;
  int tile_codes;    // the sector kernel's obs tile holds byte codes (pe_step_quad<..., BT>); so do the
                     // prefetched records' obs rows
  int obs_codes;     // pe_config.obs_codes: pe_step_codes allowed (implies tile_codes)
  const char* kname;
  char kname_buf[64];  // kname with the envs-per-workgroup suffix (small batches)
  void* cur_mem;     // CurriculumWrapper records (pe_curriculum_enable), or NULL
  size_t lds_floor;  // minimum dynamic LDS per step workgroup (PE_LDS_FLOOR, debug builds only)
  int quad_waves;    // waves per workgroup of the sector kernel (4; 8 via PE_QUAD_WAVES in debug builds)
  int quad_epb;      // envs per workgroup of the sector kernel (64; 16 / 32 for small batches, C16R6 one-word)
  int gr2;           // the two-word C16R6 kernel with the grid block in round 1 (pe_step_quad GR2)
  int stagger;       // sector-kernel start delay per block quarter (PE_STAGGER, debug builds only)
  int pipe_wpc;      // > 0: the persistent pipelined sector kernel (pe_step_pipe), this many
                     // workgroups per CU; 0: pe_step_quad
  int num_cus;       // the device's CUs (the persistent grid)
  int coop_max_done; // wave-cooperative auto-resets up to this many done envs per block (pe_coop.hpp;
                     // pe_config.coop_max_done)
  pe::Prefetch pf;   // prefetched resets (pf.scal == NULL: off)
  void* pf_mem;
  int pf_every;      // steps between queue-mode prefetch launches (pe_config.prefetch_every)
  int pf_count;      // steps since the last one
  int pf_blocks;     // queue-mode prefetch grid: workgroups resident at once
};

// pe_internal_set_error (plantos_batch.hip): records pe_last_error() for this thread.
extern "C" int pe_internal_set_error(int code, const char* msg);
// pe_internal_flush_vx (plantos_batch.hip): the steps' deferred visit-overflow writes applied
// on `stream` (before anything reads the exact visit counts, e.g. the MCTS clone).
extern "C" int pe_internal_flush_vx(const pe_handle* h, void* stream);
