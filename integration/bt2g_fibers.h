// integration/bt2g_fibers.h -- user-mode fibers for the reference's search
// workers (the drop-in's batch-first schedule; see bt2g_fibers.cpp).
#ifndef BT2G_FIBERS_H_
#define BT2G_FIBERS_H_

#include <stddef.h>

namespace bt2gf {

// The running fiber (nullptr on an ordinary thread).
void* self();

// Called by a fiber: hand `req` to the carrier's outbox (it reaches the seam
// dispatchers, through the flush hook, once every runnable fiber of the
// carrier has had its turn) and suspend until wake(self) is called for it.
void block_on(void* req);

// The same for n requests at once; the fiber resumes at the first wake(self)
// (the seam side wakes it once, when the last of them completed).
void block_on_many(void* const* reqs, size_t n);

// Resume fibers whose requests completed (any thread; grouped per carrier).
void wake_many(void* const* fibers, size_t n);

// The seam side: receives a carrier's outbox (requests in program order of
// the carrier's fibers).  Set once, before the first fiber runs.
typedef void (*FlushFn)(void* const* reqs, size_t n);
void set_flush(FlushFn fn);

// Called once on the thread that spawns the first fiber, before it runs (the
// seam side opens its GPU context and dispatchers there, on an ordinary stack).
typedef void (*InitFn)();
void set_init(InitFn fn);

// Whether the drop-in runs its workers as fibers ($BT2G_FIBERS, default on).
bool enabled();

// Fibers created so far (the server's search workers).
size_t count();

// A pointer-sized slot of the running fiber for its caller's use (nullptr on an
// ordinary thread): state that must not be shared by the fibers of a carrier.
void** local();

// $BT2G_MUTEX_PROF=<path>: contended pthread_mutex_lock call sites of fibers
// (note: the wrapper; dump: "offset count" lines, written at SIGTERM)
void mutex_prof_note(void* ra);
void mutex_prof_dump();

}  // namespace bt2gf

#endif
