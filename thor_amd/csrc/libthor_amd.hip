// Single translation unit for libthor_amd.so (no relocatable device code).
#include "recon.hip"
#include "resid.hip"
#include "txq.hip"
#include "inter.hip"
#include "intra.hip"
#include "loopfilter.hip"
#include "capi.hip"
#include "simd_surface.hip"
