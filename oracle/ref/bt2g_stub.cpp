// oracle/ref/bt2g_stub.cpp -- TEST INFRASTRUCTURE ONLY (never part of the product).
//
// A CPU stand-in for the subset of include/bt2g.h that integration/bt2g_seams.cpp
// calls, answered by the REFERENCE's own code through harness.cpp (this
// directory).  Linked into oracle/_ref/libbt2g_stub.so and from there into
// oracle/_ref/bowtie2-align-server-stub, it lets the CPU tests check the
// reference-side binding itself (RNG replay of candidate fates, AlnRes
// construction, the seed-cache protocol) on this container, where there is
// no GPU: the stub server's SAM must equal the stock server's.  The GPU build
// (bowtie2-align-server-gpu) links the real libbt2g.so instead.
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>
#include <string>
#include <vector>
#include "bt2g.h"

extern "C" {
void* bt2ref_open(const char* base);
void bt2ref_close(void* vh);
void bt2ref_exact_sweep(void* vh, int n, const char** seqs, const char** quals, int mineMax, uint64_t* out);
void bt2ref_one_mm(void* vh, int n, const char** seqs, const char** quals, const int64_t* minsc, int local, int nofw,
                   int norc, int cap, int64_t* out, int32_t* counts, uint64_t* bwops);
void bt2ref_one_mm_sc(void* vh, int n, const char** seqs, const char** quals, const int64_t* minsc, int local,
                      int nofw, int norc, int cap, int64_t* out, int32_t* counts, uint64_t* bwops, const void* sp);
void bt2ref_exact_sweep_fr(void* vh, int n, const char** seqs, const char** quals, int mineMax, int nofw, int norc,
                           uint64_t* out);
void bt2ref_seed_search(void* vh, int n, const char** seqs, const char** quals, int seedlen, int interval, int offset,
                        int maxseeds, uint32_t* out, int32_t* nseeds, uint64_t* bwops);
int bt2ref_sw(const char* seq, const char* qual, int fw, const uint8_t* rfmask, int ncol, int64_t minsc,
              const void* sp, int enable8, int cap, int64_t* out, int64_t* cands, int32_t* mat);
int bt2ref_sw_bt(const char* seq, const char* qual, int fw, const uint8_t* rfmask, int ncol, int64_t minsc,
                 const void* sp, int enable8, int triml, int corel, int corer, int maxaln, int maxedit,
                 int64_t* out, int64_t* aln, int32_t* edits, int32_t* fates, int capf);
void bt2ref_extend(void* vh, int n, const char** seqs, const char** quals, const int32_t* fw, const uint32_t* off,
                   const uint32_t* len, const uint32_t* tb, uint32_t* out);
void bt2ref_get_offsets(void* vh, int n, const uint32_t* rows, uint32_t* out);
int bt2ref_get_stretch(void* vh, uint32_t refidx, uint64_t off, uint64_t len, uint8_t* dst);
uint64_t bt2ref_ref_len(void* vh, uint32_t refidx);
void bt2ref_ungapped(void* vh, int n, const char** seqs, const char** quals, const uint8_t* fws,
                     const uint32_t* refidx, const int64_t* off, const int64_t* minsc, const void* sp,
                     int ohang, int maxedit, int64_t* out, int32_t* edits);
}

struct bt2g_ctx {
	void* ref;
	std::string base;
};

namespace {
thread_local std::string g_err;

int fail(int rc, const char* fmt, ...) {
	char buf[512];
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(buf, sizeof(buf), fmt, ap);
	va_end(ap);
	g_err = buf;
	return rc;
}

std::string ascii(const uint8_t* codes, uint32_t len) {
	std::string s(len, 'N');
	for(uint32_t i = 0; i < len; i++) s[i] = "ACGTN"[codes[i] > 4 ? 4 : codes[i]];
	return s;
}

std::string qstr(const uint8_t* q, uint32_t len) { return std::string((const char*)q, len); }

// Edit characters come back from the reference as ASCII; bt2g_mm1 carries codes.
int32_t code_of(int64_t ch) {
	switch((int)ch) { case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3; default: return 4; }
}
}  // namespace

extern "C" {

const char* bt2g_last_error(void) { return g_err.c_str(); }

int bt2g_open(const char* base, int, bt2g_ctx** out) {
	bt2g_ctx* c = new bt2g_ctx();
	c->ref = bt2ref_open(base);
	if(!c->ref) { delete c; return fail(BT2G_ERR_IO, "bt2ref_open"); }
	c->base = base;
	*out = c;
	return BT2G_OK;
}

int bt2g_set_priority(bt2g_ctx* c, int high) {
	(void)high;
	return c ? BT2G_OK : fail(BT2G_ERR_ARG, "null ctx");
}

int bt2g_set_cu_share(bt2g_ctx* c, uint32_t num, uint32_t den) {
	(void)num;
	(void)den;
	return c ? BT2G_OK : fail(BT2G_ERR_ARG, "null ctx");
}

int bt2g_open_shared(bt2g_ctx* base, bt2g_ctx** out) {
	if(!base || !out) return fail(BT2G_ERR_ARG, "null argument");
	bt2g_ctx* c = new bt2g_ctx();
	c->ref = bt2ref_open(base->base.c_str());   // the harness index is driven by one thread
	if(!c->ref) { delete c; return fail(BT2G_ERR_IO, "bt2ref_open"); }
	c->base = base->base;
	*out = c;
	return BT2G_OK;
}

int bt2g_close(bt2g_ctx* c) {
	if(c) { bt2ref_close(c->ref); delete c; }
	return BT2G_OK;
}

int bt2g_exact_sweep(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                     uint32_t mine_max, int nofw, int norc, uint32_t* out) {
	for(uint32_t i = 0; i < n; i++) {
		std::string s = ascii(reads + (size_t)i * stride, lens[i]), q(lens[i], 'I');
		const char* sp = s.c_str();
		const char* qp = q.c_str();
		uint64_t o[8];
		bt2ref_exact_sweep_fr(c->ref, 1, &sp, &qp, (int)mine_max, nofw, norc, o);
		uint32_t* w = out + 8 * (size_t)i;
		w[0] = (uint32_t)o[0]; w[1] = (uint32_t)o[1]; w[2] = (uint32_t)o[3]; w[3] = (uint32_t)o[4];
		w[4] = (uint32_t)o[5]; w[5] = (uint32_t)o[6]; w[6] = (uint32_t)o[7]; w[7] = 0;
	}
	return BT2G_OK;
}

int bt2g_one_mm(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                uint32_t n, const int32_t* minsc, const bt2g_scoring* sc, int nofw, int norc, uint32_t cap,
                bt2g_mm1* hits, int32_t* counts, uint32_t* bwops, uint32_t*) {
	int rc = BT2G_OK;
	for(uint32_t i = 0; i < n; i++) {
		std::string s = ascii(reads + (size_t)i * stride, lens[i]), q = qstr(quals + (size_t)i * stride, lens[i]);
		const char* sp = s.c_str();
		const char* qp = q.c_str();
		int64_t ms = minsc[i];
		std::vector<int64_t> o(6 * (size_t)cap + 6);
		uint64_t ops = 0;
		bt2ref_one_mm_sc(c->ref, 1, &sp, &qp, &ms, sc->local, nofw, norc, (int)cap, o.data(), &counts[i], &ops, sc);
		bwops[i] = (uint32_t)ops;
		for(int32_t k = 0; k < counts[i] && k < (int32_t)cap; k++) {
			bt2g_mm1& h = hits[(size_t)i * cap + k];
			const int64_t* x = &o[6 * (size_t)k];
			h.top = (uint32_t)x[0]; h.bot = (uint32_t)x[1]; h.fw = (int32_t)x[2]; h.score = (int32_t)x[3];
			h.pos = (int32_t)x[4]; h.chr = code_of(x[5] & 0xff); h.qchr = code_of(x[5] >> 8); h.pad = 0;
		}
		if(counts[i] > (int32_t)cap) rc = BT2G_ERR_OVERFLOW;
	}
	return rc;
}

int bt2g_exact_sweep_1mm(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                         const uint32_t* lens, uint32_t n, uint32_t mine_max, int nofw, int norc, int skip_exact,
                         const int32_t* minsc, const bt2g_scoring* sc, uint32_t cap, uint32_t* sweep,
                         bt2g_mm1* hits, int32_t* counts, uint32_t* bwops, uint32_t* mm_loads, uint32_t off_cap,
                         uint32_t* offs) {
	if(mm_loads) memset(mm_loads, 0, sizeof(uint32_t) * n);     // (the stand-in gathers no sides)
	int rc = bt2g_exact_sweep(c, reads, stride, lens, n, mine_max, nofw, norc, sweep);
	if(rc) return rc;
	for(uint32_t i = 0; i < n; i++) {
		// the gate of bt2g_one_mm_gated_dev (fm_one_mm.hip k_one_mm_items)
		const uint32_t mfw = sweep[8 * (size_t)i], mrc = sweep[8 * (size_t)i + 1];
		const bool yfw = mfw <= 1 && !nofw, yrc = mrc <= 1 && !norc;
		counts[i] = 0;
		bwops[i] = 0;
		if(((mfw < mrc ? mfw : mrc) == 0 && skip_exact) || !(yfw || yrc)) continue;
		rc = bt2g_one_mm(c, reads + (size_t)i * stride, quals + (size_t)i * stride, stride, lens + i, 1, minsc + i, sc,
		                 !yfw, !yrc, cap, hits + (size_t)i * cap, counts + i, bwops + i, nullptr);
		if(rc && rc != BT2G_ERR_OVERFLOW) return rc;
	}
	if(offs) {
		// the small ranges' rows (include/bt2g.h), by the reference's getOffset
		const size_t per = (size_t)(2 + cap) * off_cap;
		for(uint32_t i = 0; i < n; i++) {
			for(size_t k = 0; k < per; k++) offs[i * per + k] = 0xffffffffu;
			for(uint32_t slot = 0; slot < 2 + cap; slot++) {
				uint32_t top = 0, bot = 0;
				if(slot < 2) {
					if(sweep[8 * (size_t)i + slot] == 0) { top = sweep[8 * (size_t)i + 2 + 2 * slot]; bot = sweep[8 * (size_t)i + 3 + 2 * slot]; }
				} else if((int32_t)(slot - 2) < std::min<int32_t>(counts[i], (int32_t)cap)) {
					top = hits[(size_t)i * cap + slot - 2].top;
					bot = hits[(size_t)i * cap + slot - 2].bot;
				}
				if(bot <= top || bot - top > off_cap) continue;
				std::vector<uint32_t> rows(bot - top);
				for(uint32_t j = 0; j < bot - top; j++) rows[j] = top + j;
				bt2g_get_offset(c, rows.data(), (uint32_t)rows.size(), offs + i * per + (size_t)slot * off_cap, nullptr);
			}
		}
	}
	return BT2G_OK;
}

int bt2g_seed_search(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                     uint32_t seedlen, uint32_t interval, uint32_t offset, uint32_t maxseeds, uint32_t* out,
                     int32_t* nseeds, uint32_t* bwops, uint32_t*) {
	for(uint32_t i = 0; i < n; i++) {
		std::string s = ascii(reads + (size_t)i * stride, lens[i]), q(lens[i], 'I');
		const char* sp = s.c_str();
		const char* qp = q.c_str();
		uint64_t ops = 0;
		bt2ref_seed_search(c->ref, 1, &sp, &qp, (int)seedlen, (int)interval, (int)offset, (int)maxseeds,
		                   out + (size_t)i * 2 * maxseeds * 4, &nseeds[i], &ops);
		bwops[i] = (uint32_t)ops;
	}
	return BT2G_OK;
}

// bt2g_seed_search + bt2g_extend of each seed's range + the small ranges' rows
// (include/bt2g.h), each by the reference's own code
int bt2g_seed_search_ext(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                         uint32_t seedlen, uint32_t interval, uint32_t offset, uint32_t maxseeds, uint32_t* out,
                         int32_t* nseeds, uint32_t* bwops, uint32_t* loads, bt2g_ext_out* ext, uint32_t off_cap,
                         uint32_t* offs) {
	int rc = bt2g_seed_search(c, reads, stride, lens, n, seedlen, interval, offset, maxseeds, out, nseeds, bwops, loads);
	if(rc) return rc;
	for(uint32_t i = 0; i < n; i++)
		for(uint32_t f = 0; f < 2; f++)
			for(uint32_t s = 0; s < maxseeds; s++) {
				const size_t k = ((size_t)i * 2 + f) * maxseeds + s;
				const uint32_t* o = out + k * 4;
				const uint32_t L = std::min(seedlen, lens[i]), depth = s * interval + offset;
				if(ext) {
					ext[k] = bt2g_ext_out{0, 0, 0, 0};
					if(o[1] > o[0] && depth + L <= lens[i]) {
						const bt2g_ext_in q{i, f == 0 ? 1 : 0, depth, L, o[0], o[1], o[2], o[3]};
						if((rc = bt2g_extend(c, reads, stride, lens, n, &q, 1, &ext[k]))) return rc;
					}
				}
				if(offs) {
					for(uint32_t j = 0; j < off_cap; j++) offs[k * off_cap + j] = 0xffffffffu;
					if(o[1] > o[0] && o[1] - o[0] <= off_cap) {
						std::vector<uint32_t> rows(o[1] - o[0]);
						for(uint32_t j = 0; j < rows.size(); j++) rows[j] = o[0] + j;
						bt2g_get_offset(c, rows.data(), (uint32_t)rows.size(), offs + k * off_cap, nullptr);
					}
				}
			}
	return BT2G_OK;
}

int bt2g_ungapped(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                  const bt2g_ug_problem* probs, uint32_t n, const bt2g_scoring* sc, int ohang, uint32_t maxedit,
                  bt2g_ug_result* res, bt2g_edit* edits) {
	for(uint32_t i = 0; i < n; i++) {
		const bt2g_ug_problem& p = probs[i];
		std::string s = ascii(reads + (size_t)p.read * stride, lens[p.read]);
		std::string q = qstr(quals + (size_t)p.read * stride, lens[p.read]);
		const char* sp = s.c_str();
		const char* qp = q.c_str();
		uint8_t fw = p.fw ? 1 : 0;
		uint32_t ri = p.refidx;
		int64_t off = p.off, ms = p.minsc, o[10];
		std::vector<int32_t> ed(4 * (size_t)maxedit);
		bt2ref_ungapped(c->ref, 1, &sp, &qp, &fw, &ri, &off, &ms, sc, ohang, (int)maxedit, o, ed.data());
		bt2g_ug_result& r = res[i];
		memset(&r, 0, sizeof(r));
		r.ret = (int32_t)o[0]; r.score = (int32_t)o[1]; r.refoff = o[2]; r.ns = (int32_t)o[3];
		r.refns = (int32_t)o[4]; r.nedit = (int32_t)o[5]; r.trim5p = (int32_t)o[6]; r.trim3p = (int32_t)o[7];
		for(int32_t e = 0; e < r.nedit && e < (int32_t)maxedit; e++) {
			bt2g_edit& d = edits[(size_t)i * maxedit + e];
			d.pos = (uint32_t)ed[4 * e]; d.type = (uint8_t)ed[4 * e + 1]; d.chr = (uint8_t)ed[4 * e + 2];
			d.qchr = (uint8_t)ed[4 * e + 3]; d.pad = 0;
		}
	}
	return BT2G_OK;
}

int bt2g_sw_align_bt(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                     const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows, uint64_t,
                     const bt2g_sw_rect* rects, const bt2g_scoring* sc, int enable8, uint32_t cap, bt2g_sw_result* res,
                     bt2g_sw_cand* cands, uint32_t maxaln, uint32_t maxedit, int32_t* naln, bt2g_sw_aln* alns,
                     bt2g_edit* edits, int8_t* fates) {
	int rc = BT2G_OK;
	for(uint32_t i = 0; i < nprob; i++) {
		const bt2g_sw_problem& p = probs[i];
		if(!rects) return fail(BT2G_ERR_ARG, "stub: rects required");
		std::string s = ascii(reads + (size_t)p.read * stride, lens[p.read]);
		std::string q = qstr(quals + (size_t)p.read * stride, lens[p.read]);
		// the caller's window, or (win_off < 0) the reference's own bases at
		// [refl, refl + ncol], N outside the reference, as masks (initRef's window)
		std::vector<uint8_t> own;
		const uint8_t* rf = windows + p.win_off;
		if(p.win_off < 0) {
			own.assign((size_t)p.ncol + 1, 16);
			const int64_t rl = (int64_t)bt2ref_ref_len(c->ref, p.refidx);
			for(uint32_t j = 0; j <= p.ncol; j++) {
				const int64_t pos = p.refl + (int64_t)j;
				if(pos >= 0 && pos < rl) {
					uint8_t b;
					bt2ref_get_stretch(c->ref, p.refidx, (uint64_t)pos, 1, &b);
					own[j] = (uint8_t)(1u << (b > 4 ? 4 : b));
				}
			}
			rf = own.data();
		}
		int64_t o[7];
		std::vector<int64_t> cc(3 * (size_t)cap + 3);
		bt2ref_sw(s.c_str(), q.c_str(), p.fw, rf, (int)p.ncol, p.minsc, sc, enable8, (int)cap, o, cc.data(), nullptr);
		bt2g_sw_result& r = res[i];
		r.aligned = (int32_t)o[0];
		r.best = o[1] < INT32_MIN ? INT32_MIN : (int32_t)o[1];
		r.u8succ = (int32_t)o[2]; r.i16succ = (int32_t)o[3]; r.colstop = (int32_t)o[4];
		r.lastsolcol = (int32_t)o[5]; r.ncand = (int32_t)o[6]; r.flag = 0;
		for(int64_t k = 0; k < o[6] && k < (int64_t)cap; k++) {
			bt2g_sw_cand& d = cands[(size_t)i * cap + k];
			d.row = (int32_t)cc[3 * k]; d.col = (int32_t)cc[3 * k + 1]; d.score = (int32_t)cc[3 * k + 2];
		}
		if(o[6] > (int64_t)cap) { rc = BT2G_ERR_OVERFLOW; continue; }
		std::vector<int64_t> al(10 * (size_t)maxaln);
		std::vector<int32_t> ed(4 * (size_t)maxaln * maxedit);
		std::vector<int32_t> ft((size_t)cap, 0);
		int64_t o2[7];
		const bt2g_sw_rect& rc0 = rects[i];
		int na = bt2ref_sw_bt(s.c_str(), q.c_str(), p.fw, rf, (int)p.ncol, p.minsc, sc, enable8, rc0.triml, rc0.corel,
		                      rc0.corer, (int)maxaln, (int)maxedit, o2, al.data(), ed.data(), ft.data(), (int)cap);
		naln[i] = na < (int)maxaln ? na : (int)maxaln;
		for(int k = 0; k < naln[i]; k++) {
			bt2g_sw_aln& a = alns[(size_t)i * maxaln + k];
			const int64_t* x = &al[10 * (size_t)k];
			a.cand = (int32_t)x[0]; a.score = (int32_t)x[1]; a.off = (int32_t)x[2]; a.ns = (int32_t)x[4];
			a.gaps = (int32_t)x[5]; a.refns = (int32_t)x[6]; a.nedit = (int32_t)x[7]; a.trim5p = (int32_t)x[8];
			a.trim3p = (int32_t)x[9]; a.pad = 0;
			for(int32_t e = 0; e < a.nedit && e < (int32_t)maxedit; e++) {
				const int32_t* y = &ed[4 * ((size_t)k * maxedit + e)];
				bt2g_edit& d = edits[((size_t)i * maxaln + k) * maxedit + e];
				d.pos = (uint32_t)y[0]; d.type = (uint8_t)y[1]; d.chr = (uint8_t)y[2]; d.qchr = (uint8_t)y[3]; d.pad = 0;
			}
		}
		// fates: the reference marks candidates it never reached with 0; only
		// those up to the maxaln-th success are meaningful, as for the engine
		if(fates)
			for(uint32_t k = 0; k < cap; k++) fates[(size_t)i * cap + k] = (int8_t)ft[k];
	}
	return rc;
}

int bt2g_extend(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t nreads,
                const bt2g_ext_in* in, uint32_t n, bt2g_ext_out* out) {
	for(uint32_t i = 0; i < n; i++) {
		const bt2g_ext_in& q = in[i];
		if(q.read >= nreads) return fail(BT2G_ERR_ARG, "stub: bad read");
		std::string s = ascii(reads + (size_t)q.read * stride, lens[q.read]);
		std::string qq(lens[q.read], 'I');
		const char* sp = s.c_str();
		const char* qp = qq.c_str();
		uint32_t tb[4] = {q.topf, q.botf, q.topb, q.botb}, o[3];
		bt2ref_extend(c->ref, 1, &sp, &qp, &q.fw, &q.off, &q.len, tb, o);
		out[i].nlex = o[0]; out[i].nrex = o[1]; out[i].fmops = o[2]; out[i].loads = 0;
	}
	return BT2G_OK;
}

int bt2g_get_offset(bt2g_ctx* c, const uint32_t* rows, uint32_t n, uint32_t* offs, uint32_t* loads) {
	bt2ref_get_offsets(c->ref, (int)n, rows, offs);
	if(loads) memset(loads, 0, sizeof(uint32_t) * n);
	return BT2G_OK;
}

// the packed flavour (include/bt2g.h): the unpacked call, then packed here
int bt2g_sw_align_bt_packed(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                            const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob,
                            const uint8_t* windows, uint64_t wl, const bt2g_sw_rect* rects, const bt2g_scoring* sc,
                            int enable8, uint32_t cap, bt2g_sw_result* res, uint32_t maxaln, uint32_t maxedit,
                            int32_t* naln, bt2g_sw_aln* alns, bt2g_sw_cand* cands, int8_t* fates, bt2g_edit* edits,
                            uint64_t* totals) {
	std::vector<bt2g_sw_cand> C((size_t)nprob * cap);
	std::vector<int8_t> F((size_t)nprob * cap);
	std::vector<bt2g_edit> E((size_t)nprob * maxaln * maxedit);
	int rc = bt2g_sw_align_bt(c, reads, quals, stride, lens, probs, nprob, windows, wl, rects, sc, enable8, cap, res,
	                          C.data(), maxaln, maxedit, naln, alns, E.data(), F.data());
	if(rc && rc != BT2G_ERR_OVERFLOW) return rc;
	uint64_t tc = 0, ta = 0, te = 0;
	for(uint32_t i = 0; i < nprob; i++) {
		const uint32_t nc = (uint32_t)std::min<int64_t>(std::max<int32_t>(res[i].ncand, 0), cap);
		for(uint32_t k = 0; k < nc; k++, tc++) {
			cands[tc] = C[(size_t)i * cap + k];
			if(fates) fates[tc] = F[(size_t)i * cap + k];
		}
		const uint32_t na = (uint32_t)std::min<int64_t>(std::max<int32_t>(naln[i], 0), maxaln);
		ta += na;
		for(uint32_t k = 0; k < na; k++) {
			const uint32_t ne = (uint32_t)std::min<int64_t>(std::max<int32_t>(alns[(size_t)i * maxaln + k].nedit, 0), maxedit);
			for(uint32_t e = 0; e < ne; e++) edits[te++] = E[((size_t)i * maxaln + k) * maxedit + e];
		}
	}
	totals[0] = tc;
	totals[1] = ta;
	totals[2] = te;
	return rc;
}

// kernel timing: nothing runs on a device here
int bt2g_set_profiling(bt2g_ctx*, int) { return BT2G_OK; }

int bt2g_kernel_stats(bt2g_ctx*, int, uint64_t* launches, double* total_ms) {
	if(launches) *launches = 0;
	if(total_ms) *total_ms = 0;
	return BT2G_OK;
}

}  // extern "C"
