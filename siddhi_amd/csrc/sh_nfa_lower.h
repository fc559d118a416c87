// sh_nfa_lower.h — host lowering of sh_app_desc into the general engine's
// NFA table (sh_nfa_lower.cpp).
#pragma once
#include <string>

#include "sh_nfa.h"

// 0 ok, -1 unsupported (err says why)
int nf_lower(const sh_app_desc* app, nf_table* T, std::string* err);
// (re)computes every query's per-key layout and the key block size
void nf_set_caps(nf_table* T, int list_cap, int se_cap, int node_cap, int hold_cap, int sched_cap,
                 int group_cap = 4);
