// integration/bt2g_batch_conn.cpp -- the batch server's read buffers per
// client connection.
//
// The reference gives a connection 4 x nthreads + 1 read buffers of 16 reads
// (PatternSourceServiceFactory::align, pat.cpp:2045-2050), each built with its
// Read objects when the connection opens and freed when it closes: a worker
// held a buffer until its 16 reads were aligned.  The batch driver copies a
// buffer's reads into its slots and returns the buffer at once
// (bt2g_batch.cpp), so a few buffers keep a connection's reads flowing, and
// the rest were only allocation churn on the connection's thread (each
// connection made and freed ~65 x 16 x 2 Reads at -p 16).  $BT2G_READAHEAD
// sets a smaller depth; by default the reference's (r04q: 16 buffers starved
// the drivers -- ~400 reads in flight per driver against ~640 with 65).
#include <pthread.h>
#include <stdlib.h>
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

extern "C" bool bt2g_real__ZN27PatternSourceServiceFactory5alignEil(PatternSourceServiceFactory* self, int fd,
                                                                   long data_size);

bool PatternSourceServiceFactory::align(int fd, long data_size) {
	// set once, by the first connection, before any connection reads the member
	// (the member is const in pat.h and read through `this` at every connection)
	static std::once_flag once;
	std::call_once(once, [this] {
		unsigned int depth = n_readahead_;
		if(const char* e = getenv("BT2G_READAHEAD"))
			if(atol(e) > 0) depth = (unsigned int)atol(e);
		if(depth < n_readahead_) const_cast<unsigned int&>(n_readahead_) = depth;
	});
	return bt2g_real__ZN27PatternSourceServiceFactory5alignEil(this, fd, data_size);
}
