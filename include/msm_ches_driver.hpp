// msm_ches_driver.hpp -- the reference's driver-level API (ref main_p1.cpp /
// main_p2.cpp: globals :41-50, init_* :52-178, the four timed MSM methods
// :192-436, test_pippengers :438-610) on top of libmsm_mi355x.so.
//
// Same function names, argument meaning and return values as the reference
// driver; the compile-time configuration of ref ches_config_files/*.h
// (N_EXP, q, h, ...) and makefile `group=` become run-time arguments of
// msm_driver_configure().  One group per translation unit, as in the reference
// (main_p1 / main_p2): define MSM_DRIVER_GROUP to 1 (G1, blst_p1_affine) or 2
// (G2, blst_p2_affine) before including.
//
// Differences from the reference, all deliberate:
//  * PRECOMPUTATION_POINTS_LIST_3nh / _BGMW95 live in HBM (device contexts);
//    the host globals stay NULL unless msm_driver_configure(..., host_tables=1)
//    asks for blst-layout host copies (byte-identical to the reference's).
//  * Scalars for test_pippengers come from the seeded SplitMix64 generator
//     instead of OpenSSL RAND_bytes, so runs are repeatable.
//  * The CHES results are the exact sums (the last-element guard defect of
//    ref multi_scalar.c:461 is not reproduced).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "msm_mi355x.h"

#ifndef MSM_DRIVER_GROUP
#define MSM_DRIVER_GROUP 1
#endif
#if MSM_DRIVER_GROUP == 1
typedef blst_p1_affine msm_driver_affine;
#else
typedef blst_p2_affine msm_driver_affine;
#endif

// layout of the reference's numeric::uint256_t (src_from_aztec/numeric/uint256/
// uint256.hpp): four 64-bit limbs, least significant first == a 32-byte LE scalar
struct uint256_t {
  uint64_t data[4];
};

// ref main_p1.cpp:41-50 (plus the configuration macros of ches_config_files)
extern int N_EXP;
extern size_t N_POINTS;
extern int q_RADIX_EXP, h_LEN_SCALAR, a_LEADING_TERM, B_SIZE, EXPONENT_OF_q_BGMW95, h_BGMW95;
extern digit_decomposition *DIGIT_CONVERSION_HASH_TABLE;
extern int *BUCKET_SET;
extern int *BUCKET_VALUE_TO_ITS_INDEX;
extern msm_driver_affine *FIX_POINTS_LIST;
extern msm_driver_affine *PRECOMPUTATION_POINTS_LIST_3nh;
extern msm_driver_affine *PRECOMPUTATION_POINTS_LIST_BGMW95;

// the ches_config_files/config_file_n_exp_<n_exp>[_beta].h selection; returns 0 or an MSM_E* code
int msm_driver_configure(int n_exp, int beta, int device, int host_tables);

void init_fix_point_list();                  // ref main_p1.cpp:52-66
void free_init_fix_point_list();
void init_pippenger_CHES_q_over_5();         // ref main_p1.cpp:128-178 (table built on the GPU)
void free_init_pippenger_CHES_q_over_5();
void init_pippenger_BGMW95();                // ref main_p1.cpp:94-122
void free_init_pippenger_BGMW95();

msm_driver_affine pippenger_variant_q_over_5_CHES(uint256_t scalars_array[]);                       // :192-246
msm_driver_affine pippenger_variant_q_over_5_CHES_integral_scalar_conversion(uint256_t scalars_array[]);  // :249-291
msm_driver_affine pippenger_variant_BGMW95(uint256_t scalars_array[]);                              // :294-398
msm_driver_affine pippenger_blst_built_in(uint256_t scalars_array[]);                               // :400-436

// ref main_p1.cpp:438-610: TEST_NUM scalar arrays x LOOP_NUM repetitions of the four
// methods, mean times, results, improvement percentages; returns 0 iff all four
// methods agree on every array
int test_pippengers();
