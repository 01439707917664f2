// integration/bt2g_gw_spec.h -- force-included (-include) when the drop-in
// compiles the reference's aligner_sw_driver.cpp.
//
// Declares that the two members of GroupWalk2S<TSlice, 16> that SwDriver calls
// -- init (group_walk.h:1105-1140) and advanceElement (group_walk.h:1161-1216)
// -- are explicitly specialised elsewhere (integration/bt2g_seams.cpp), so the
// compiler emits calls to them instead of instantiating the reference's LF
// walk.  The specialisations return exactly what the walk returns -- the
// joined-text offset of SA row topf + elt, Ebwt::getOffset (bt2_idx.cpp:150-171)
// -- resolved in batches on the GPU (bt2g_get_offset).  The reference source is
// not modified; this is a compile flag of the drop-in build only.
#pragma once
#include "aligner_cache.h"
#include "group_walk.h"

template <>
void GroupWalk2S<TSlice, 16>::init(const Ebwt& ebwtFw, const BitPairReference& ref, SARangeWithOffs<TSlice>& sa,
                                   RandomSource& rnd, WalkMetrics& met);
template <>
bool GroupWalk2S<TSlice, 16>::advanceElement(TIndexOffU elt, const Ebwt& ebwtFw, const BitPairReference& ref,
                                             SARangeWithOffs<TSlice>& sa, GroupWalkState& gws, WalkResult& res,
                                             WalkMetrics& met, PerReadMetrics& prm);
