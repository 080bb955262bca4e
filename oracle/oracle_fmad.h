/*
 * oracle_fmad.h -- the FMA contraction models of the CPU oracle (see the header of oracle.c).
 * TEST INFRASTRUCTURE ONLY.
 */
#ifndef ORACLE_FMAD_H
#define ORACLE_FMAD_H
#include <math.h>

#ifndef ORC_FMAD
#define ORC_FMAD 0
#endif
/* a*b + c*d, both products single-use: the contraction site whose fused product is a choice. */
#if ORC_FMAD == 1
#define SUM2(a, b, c, d) fmaf((a), (b), (c) * (d))
#elif ORC_FMAD == 2
#define SUM2(a, b, c, d) fmaf((c), (d), (a) * (b))
#else
#define SUM2(a, b, c, d) ((a) * (b) + (c) * (d))
#endif
/* a*b + c with an unambiguous fused product (models 1 and 2 agree). */
#if ORC_FMAD
#define FMA(a, b, c) fmaf((a), (b), (c))
#else
#define FMA(a, b, c) ((a) * (b) + (c))
#endif
/* The float value handed to an atomicAdd: rounded on its own (an opaque register barrier keeps
 * the contracting builds from fusing it into the accumulation). */
static inline float orc_rounded(float x) {
#if ORC_FMAD
    __asm__("" : "+x"(x));
#endif
    return x;
}

#endif
