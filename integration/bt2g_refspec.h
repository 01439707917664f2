// integration/bt2g_refspec.h -- reference-side definitions shared by the two
// bindings (bt2g_seams.cpp, the fiber drop-in; bt2g_batch.cpp, the batch-first
// driver).  Include from exactly one translation unit per binary: it defines
// AlignmentCache::addOnTheFlyImpl, whose reference definition the Makefile
// makes weak (weaken.sh on aligner_cache.o).
//
// AlignmentCache::addOnTheFlyImpl (aligner_cache.cpp:55-104) registers a seed
// hit's SA range in the current-read cache and appends one OFF_MASK offset slot
// per row to salist_ -- one PList::add per row in the reference; on an
// hg38-scale genome a seed in a repeat family has a range of 10^5 rows, and
// every worker's 20 MB pool gets written (r03f: the loop was 18 % of the
// drop-in's host CPU).  The slots' contents are read by GroupWalk2S alone
// (group_walk.h:368-372, 508), whose init / advanceElement the bindings
// specialise: init writes OFF_MASK over exactly the rows of the range it is
// handed, so here the slots are only reserved.  Reserving keeps the
// reference's pool use and failure point: PList::ensure(pool, 1) wherever the
// reference's add() of that row would take a page (or fail), the rest of the
// page by the count.
#ifndef BT2G_REFSPEC_H_
#define BT2G_REFSPEC_H_

#include <algorithm>
#include "aligner_cache.h"

namespace bt2gref {

struct TSAListFill : public PList<TIndexOffU, CACHE_PAGE_SZ> {
	// the effect of n calls of add(p, v) on the pool and the list's length,
	// without writing the slots: returns how many were added
	size_t reserve(Pool& p, size_t n) {
		const size_t per = (size_t)CACHE_PAGE_SZ / sizeof(TIndexOffU);
		size_t done = 0;
		while(done < n) {
			if(!ensure(p, 1)) return done;
			if(cur_ == per) {
				cur_ = 0;
				curPage_++;
			}
			const size_t k = std::min(per - cur_, n - done);
			cur_ += k;
			done += k;
		}
		return done;
	}
	// slots [i, i + n) set to v, a page at a time
	void fill(size_t i, size_t n, TIndexOffU v) {
		const size_t per = (size_t)CACHE_PAGE_SZ / sizeof(TIndexOffU);
		while(n) {
			const size_t pg = i / per, off = i % per, k = std::min(per - off, n);
			std::fill(pages_[pg] + off, pages_[pg] + off + k, v);
			i += k;
			n -= k;
		}
	}
};

// the slice's list and position (protected in PListSlice)
struct TSliceAcc : public TSlice {
	void fill(TIndexOffU v) {
		if(len_) static_cast<TSAListFill*>(list_)->fill(i_, len_, v);
	}
};

}  // namespace bt2gref

bool AlignmentCache::addOnTheFlyImpl(QVal& qv, const SAKey& sak, TIndexOffU topf, TIndexOffU botf, TIndexOffU topb,
                                     TIndexOffU botb) {
	(void)botb;
	bool added = true;
	if(!qv.valid()) qv.init((uint32_t)qlist_.size(), 0, 0);
	qv.addRange(botf - topf);
	if(!qlist_.add(pool(), sak)) return false;
	SANode* s = samap_.add(pool(), sak, &added);
	if(s == NULL) return false;
	if(added) {
		s->payload.i = (TIndexOffU)salist_.size();
		s->payload.len = botf - topf;
		s->payload.topf = topf;
		s->payload.topb = topb;
		const size_t n = botf - topf;
		const size_t k = static_cast<bt2gref::TSAListFill&>(salist_).reserve(pool(), n);
		if(k < n) {
			s->payload.len = (TIndexOffU)k;
			return false;
		}
	}
	return true;
}

#endif  // BT2G_REFSPEC_H_
