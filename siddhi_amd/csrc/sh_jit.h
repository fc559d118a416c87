// sh_jit.h — hipRTC specialisation of the window engine (sh_jit.cpp), host side.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "sh_program.h"

struct shj_window {
    const void* code;     // gfx950 code object (owned by the process-wide cache)
    size_t code_size;
    void* match;          // hipFunction_t shj_match (after shj_window_load)
    void* place;          // hipFunction_t shj_place
    void* count;          // hipFunction_t shj_count (consumer-side walk), NULL when the filter has no such form
    void* emit;           // hipFunction_t shj_emit
};

// generated source for a window-shaped program (0), -1 if it has no straight-line form
int shj_window_source(const shp_program* hp, std::string* src);
// compile only (no device needed); cached per distinct source for the process
int shj_window_compile(const shp_program* hp, shj_window* out, std::string* err);
// compile + load the module on the current device
int shj_window_load(const shp_program* hp, shj_window* out, std::string* err);
// grid of the XCD-major tile mapping for n events; returns the workgroup count
unsigned shj_tiles(int64_t n, uint32_t* tiles_per_xcd, uint32_t* ntiles);
int shj_tile_size(void);
// the bucketed matcher's consumer limit per pass (events; SH_BK_CH)
int shj_bucket_chunk(void);

// bucketed window engine matcher (shb_match); ms_attrs: stream attributes the
// match stream carries (e1-side select values), in match-stream column order
struct shj_bucket {
    void* match;          // hipFunction_t shb_match
    int n_staged;         // columns the partition moves into bucket order
    int staged_attr[4];
};
int shj_bucket_load(const shp_program* hp, const int* ms_attrs, int n_ms, shj_bucket* out, std::string* err);
int shj_bucket_source(const shp_program* hp, const int* ms_attrs, int n_ms, std::string* src);
int shj_bucket_compile(const shp_program* hp, const int* ms_attrs, int n_ms, std::string* err);
