// dis_experiments.h -- fence around the measurement-only knock-out switches.
//
// The DIS_EXP_* macros below select builds that compute WRONG values on
// purpose (a stage replaced by a constant, a load or store removed, a launch
// skipped) so that an A/B can price that stage. A product
// library must never carry one: defining any of them is an error unless the
// build also defines DIS_EXPERIMENTS, which the Makefile's default build never
// does (tools/build_variants.sh adds it for knock-out variants only).
// tests/test_experiments_fence.py checks that every DIS_EXP_* token in csrc/
// is listed here.
#pragma once

#if !defined(DIS_EXPERIMENTS) &&                                                                            \
    (defined(DIS_EXP_SKIP_HEAD) || defined(DIS_EXP_SPLIT0) || defined(DIS_EXP_FULLITERS) ||                \
     defined(DIS_EXP_NO_FB) || defined(DIS_EXP_NOREGIONLOAD) || defined(DIS_EXP_NOTILELOAD) ||             \
     defined(DIS_EXP_TAPBANKS) || defined(DIS_EXP_PYR_NOLOAD) || defined(DIS_EXP_PYR_RAWSQRT) ||           \
     defined(DIS_EXP_PYR_NOSTORE) || defined(DIS_EXP_PYR_NOSMALLSTORE) || defined(DIS_EXP_PYR_LOADONLY) || \
     defined(DIS_EXP_OUT_NODENSE) || defined(DIS_EXP_OUT_NOUPS))
#error "DIS_EXP_* knock-out switches compute wrong values: define DIS_EXPERIMENTS to build a measurement variant"
#endif

#ifdef DIS_EXPERIMENTS
#define DIS_BUILD_KIND "experiment"
#else
#define DIS_BUILD_KIND "product"
#endif
