// Wrong-result diagnostic switches -- timing ablations and stage knock-outs for
// A/B builds (scripts/build_variant.sh).  Never part of the product library:
// this header refuses to compile unless the build defines MZGO_DIAG_BUILD, and
// mzgo_common.hpp refuses any of the switches without it, so a stray -D cannot
// silently change libmzgo.so's results.
#pragma once
#ifndef MZGO_DIAG_BUILD
#error "mzgo_diag.hpp belongs to diagnostic builds only (-DMZGO_DIAG_BUILD, scripts/build_variant.sh)"
#endif

// k_tconv_ks: no LDS-DMA after the first k-step / no step barriers (wrong results)
#ifdef MZGO_TCONV_ABL_NODMA
constexpr bool kAblNoDma = true;
#else
constexpr bool kAblNoDma = false;
#endif
#ifdef MZGO_TCONV_ABL_NOBAR
constexpr bool kAblNoBar = true;
#else
constexpr bool kAblNoBar = false;
#endif

