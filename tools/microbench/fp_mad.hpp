// Montgomery product bodies with explicitly issued v_mad_u64_u32 (gfx950 device code only).
//
// Why (measured, tools/microbench/mad_chain.hip, profiles/r02_mad_chain.json): with one resident wave per
// SIMD a wave issues v_mad_u64_u32 every ~10 SIMD cycles when consecutive MADs write the same carry-out SGPR
// pair -- which is what the compiler emits for every unused carry-out -- but every ~7 cycles when the
// carry-out pairs rotate and consecutive MADs belong to independent accumulation chains.  The generated
// bodies (fp_mad_gen.hpp, gen_fp_mad.py) keep the arithmetic of fp.hpp's fp_mul_body / fp_sqr_body
// (same 28-bit-limb product scanning, same bounds) but issue each column as TWO independent chains -- the
// a*b products and the m*p products -- interleaved, with the carry-out SGPR pair rotating over four pairs;
// the two column sums are added once per column.
#pragma once
#include "fp_mad_gen.hpp"
