// integration/bt2g_server.cpp -- read-ahead depth of the server under fibers.
//
// The reference server gives every client connection 4 x nthreads + 1 read
// buffers (bt2_search.cpp:4859, PatternSourceServiceFactory::align,
// pat.cpp:2030-2050): each a PatternSourcePerThread holding 2 x 16 Read
// objects, constructed when the connection opens and destroyed when it ends.
// The rule assumes -p is the core count (16 -> 65 buffers per connection).
// The drop-in runs thousands of workers as fibers (bt2g_fibers.cpp), and
// with -p 2048 every 10 000-read connection built and freed 8 193 buffers
// (262 k Read objects) -- per read more allocator work than the alignment's,
// and the frees of blocks the fibers grew on other threads' heaps contend for
// those heaps' locks (r03i: the connection threads held 20 of the server's 69
// CPU seconds, mprotect + malloc + lock waits ~30 % of the carriers').
//
// A buffer feeds one worker at a time, so nthreads + 1 buffers let one
// connection alone keep every worker busy -- the minimum the reference's own
// comment asks for (bt2_search.cpp:4858).  But every connection builds all of
// them up front, and a 10 000-read connection at --reads-per-batch 4 uses at
// most 2 500: with 4 096 workers the unused ones were most of the server's
// allocator traffic.  Since notify_all wakes waiting fibers one after another
// (bt2g_fibers.cpp), workers waiting for buffers are cheap, and with several
// connections in flight (the benchmark protocol runs 8) nthreads / 4 + 1 per
// connection keeps them busy: r03aa/r03ab at 3.1 Gbp, 4 096 workers, 1 025 vs
// 4 097 buffers 61.5k vs 58.1k and 63.2k vs 60.8k reads/s, host CPU 55 vs 75
// s.  (One client alone gets a quarter of the workers.)  $BT2G_READAHEAD
// overrides; never more than the reference's own number.  Which buffer a batch lands in
// does not change any alignment (each read's RNG is seeded from the read
// itself), so the SAM is the stock server's -- the SAM-parity tests check it.
//
// Mechanism: pat.o is linked with PatternSourceServiceFactory::align weak
// (weaken.sh; its caller serveConnection is in the same object) and this file
// defines it: set the connection's depth, then run the reference's align
// through its bt2g_real_ alias.  The member is private and const in pat.h;
// this file alone opens the class's access to write it before the connection
// starts (the object lives on multiseedSearch's stack, writable memory).
#include <stdlib.h>
// every system header pat.h pulls in, parsed before the access override
#include <pthread.h>
#include <unistd.h>
#include <zlib.h>
#include <algorithm>
#include <array>
#include <atomic>
#include <cassert>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <limits>
#include <map>
#include <mutex>
#include <queue>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

#define private public
#define protected public
#include "pat.h"
#undef private
#undef protected

#include "bt2g_fibers.h"

extern "C" bool bt2g_real__ZN27PatternSourceServiceFactory5alignEil(PatternSourceServiceFactory* self, int fd,
                                                                   long data_size);

bool PatternSourceServiceFactory::align(int fd, long data_size) {
	// Set once, by the first connection, before it reads the member (the workers
	// exist by then: the server accepts connections after spawning them).  The
	// member is const in pat.h; it is read through `this` at every connection
	// (pat.cpp's align), never folded: the one write here is what changes it.
	static std::once_flag once;
	std::call_once(once, [this] {
		unsigned int depth = n_readahead_;
		if(const char* e = getenv("BT2G_READAHEAD")) {
			if(atol(e) > 0) depth = (unsigned int)atol(e);
		} else if(bt2gf::enabled() && bt2gf::count() > 0) {
			const size_t n = bt2gf::count();
			depth = (unsigned int)std::max(n / 4 + 1, std::min<size_t>(n + 1, 64));   // (few workers: all of them)
		}
		if(depth < n_readahead_) const_cast<unsigned int&>(n_readahead_) = depth;
	});
	return bt2g_real__ZN27PatternSourceServiceFactory5alignEil(this, fd, data_size);
}
