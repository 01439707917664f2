// tests/fibers/fiber_stress.cpp -- TEST INFRASTRUCTURE: stress of the fiber
// scheduler (integration/bt2g_fibers.cpp) under the traffic the drop-in puts
// on it.  Built by tests/test_fibers.py with the same --wrap options as the
// drop-in; with -DBT2GF_R03W against the round-3 scheduler.  Two loads:
//
//   queue  thousands of fiber workers waiting on one condition variable of a
//          ready queue (LockedQueueCV::pop, pat.h:1996-2002), OS threads
//          pushing into it with notify_all (pat.h:1981-1985), the fibers
//          re-taking the queue's mutex through the yielding
//          pthread_mutex_lock wrapper and passing the notify_all baton;
//   relay  tokens handed from fiber to fiber: each fiber waits on its own
//          mailbox (mutex + condition variable) and passes the token to
//          another fiber's with notify_one -- wake_many called from fibers on
//          every carrier at once, contending on the carriers' inbox locks
//          (r03w: the path that crashed the round-3 server).
//
// Exits 0 once `items` items were consumed; a fiber resumed while it runs
// (a double wake) aborts.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>
#include "bt2g_fibers.h"

static std::atomic<long> consumed{0};
static long target = 200000;

static void done_one() {
	if(++consumed >= target) {
		fflush(stdout);
		_exit(0);
	}
}

// ---- queue ----
static std::mutex q_mu;
static std::condition_variable q_cv;
static std::deque<int> q;
static std::mutex side_mu[4];
static std::condition_variable side_cv[4];

static void queue_worker(void* arg) {
	const long id = (long)(intptr_t)arg;
	for(;;) {
		int item;
		{
			std::unique_lock<std::mutex> lk(q_mu);
			q_cv.wait(lk, [] { return !q.empty(); });
			item = q.front();
			q.pop_front();
		}
		std::mutex& m = side_mu[(item + id) & 3];
		{
			std::lock_guard<std::mutex> g(m);
			side_cv[(item + id) & 3].notify_all();
		}
		done_one();
	}
}

// ---- relay ----
struct Mailbox {
	std::mutex mu;
	std::condition_variable cv;
	int tokens = 0;
};
static Mailbox* boxes = nullptr;
static int nboxes = 0;

static void relay_worker(void* arg) {
	const long id = (long)(intptr_t)arg;
	Mailbox& me = boxes[id];
	uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(id + 1);
	for(;;) {
		{
			std::unique_lock<std::mutex> lk(me.mu);
			me.cv.wait(lk, [&] { return me.tokens > 0; });
			me.tokens--;
		}
		x ^= x << 13;
		x ^= x >> 7;
		x ^= x << 17;
		Mailbox& to = boxes[x % (uint64_t)nboxes];
		{
			std::lock_guard<std::mutex> lk(to.mu);
			to.tokens++;
		}
		to.cv.notify_one();
		done_one();
	}
}

static void noflush(void* const*, size_t) {}

int main(int argc, char** argv) {
	const char* mode = argc > 1 ? argv[1] : "queue";
	const int nfib = argc > 2 ? atoi(argv[2]) : 2000;
	const int nprod = argc > 3 ? atoi(argv[3]) : 4;     // queue: producer threads; relay: tokens
	target = argc > 4 ? atol(argv[4]) : 200000;
	bt2gf::set_flush(noflush);
	if(!strcmp(mode, "relay")) {
		nboxes = nfib;
		boxes = new Mailbox[nfib];
		for(int i = 0; i < nprod; i++) boxes[i % nfib].tokens++;
		for(int i = 0; i < nfib; i++) {
			std::thread t(relay_worker, (void*)(intptr_t)i);    // a void(*)(void*) worker: a fiber
			t.detach();
		}
		for(;;) std::this_thread::sleep_for(std::chrono::seconds(1));
	}
	std::vector<std::thread> th;
	for(int i = 0; i < nfib; i++) {
		std::thread t(queue_worker, (void*)(intptr_t)i);
		t.detach();
	}
	// the producers: batches pushed with notify_all, as the server's connection threads do
	for(int p = 0; p < nprod; p++)
		th.emplace_back([p] {
			for(int k = 0;; k++) {
				{
					std::lock_guard<std::mutex> lk(q_mu);
					for(int j = 0; j < 16; j++) q.push_back(k * 16 + j);
				}
				q_cv.notify_all();
				if((k & 63) == 0) std::this_thread::sleep_for(std::chrono::microseconds(50 + p));
			}
		});
	for(std::thread& t : th) t.join();
	return 1;
}
