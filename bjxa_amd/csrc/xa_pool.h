/*
 * xa_pool.h -- a fixed pool of host copy threads (internal), shared by the
 * many-file path (xa_files.hip) and the host-pointer decode's output slabs
 * (xa_gpu.hip duplex_decode).
 */
#ifndef BJXA_XA_POOL_H
#define BJXA_XA_POOL_H

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

namespace xa_pool {

/* one contiguous host copy */
struct piece {
	uint8_t *to;
	const uint8_t *from;
	size_t len;
};

/*
 * Fixed pool of copy threads.  run() splits a list of pieces into equal
 * byte shares (cutting pieces where needed), one per worker plus the
 * calling thread, and returns when every share is copied.
 */
class copy_pool {
public:
	/* n workers, or as many as could be started (a share per started
	 * worker; with none the calling thread copies everything) */
	explicit copy_pool(unsigned n) : n_(0)
	{
		try {
			th_.reserve(n);
			for (unsigned i = 0; i < n; i++) {
				th_.emplace_back([this, i] { work(i + 1); });
				n_++;
			}
		} catch (...) {
		}
	}
	~copy_pool()
	{
		{
			std::lock_guard<std::mutex> l(m_);
			quit_ = true;
		}
		cv_.notify_all();
		for (auto &t : th_)
			t.join();
	}
	void run(const std::vector<piece> &p)
	{
		size_t total = 0;
		for (const piece &x : p)
			total += x.len;
		if (total == 0)
			return;
		/* small jobs on the calling thread only */
		if (n_ == 0 || total < ((size_t)4 << 20)) {
			for (const piece &x : p)
				memcpy(x.to, x.from, x.len);
			return;
		}
		{
			std::lock_guard<std::mutex> l(m_);
			job_ = &p;
			total_ = total;
			pending_ = n_;
			gen_++;
		}
		cv_.notify_all();
		share(p, total, 0);
		std::unique_lock<std::mutex> l(m_);
		done_.wait(l, [this] { return pending_ == 0; });
		job_ = NULL;
	}

private:
	/* copy bytes [k*total/(n+1), (k+1)*total/(n+1)) of the piece list */
	void share(const std::vector<piece> &p, size_t total, unsigned k)
	{
		const size_t lo = total / (n_ + 1) * k;
		const size_t hi = k == n_ ? total : total / (n_ + 1) * (k + 1);
		size_t at = 0;
		for (const piece &x : p) {
			const size_t a = std::max(lo, at), b = std::min(hi,
			    at + x.len);
			if (a < b)
				memcpy(x.to + (a - at), x.from + (a - at), b - a);
			at += x.len;
			if (at >= hi)
				break;
		}
	}
	void work(unsigned k)
	{
		unsigned long seen = 0;
		for (;;) {
			const std::vector<piece> *p;
			size_t total;
			{
				std::unique_lock<std::mutex> l(m_);
				cv_.wait(l, [&] { return quit_ || gen_ != seen; });
				if (quit_)
					return;
				seen = gen_;
				p = job_;
				total = total_;
			}
			share(*p, total, k);
			std::lock_guard<std::mutex> l(m_);
			if (--pending_ == 0)
				done_.notify_one();
		}
	}
	unsigned n_;
	std::vector<std::thread> th_;
	std::mutex m_;
	std::condition_variable cv_, done_;
	const std::vector<piece> *job_ = NULL;
	size_t total_ = 0;
	unsigned pending_ = 0;
	unsigned long gen_ = 0;
	bool quit_ = false;
};

/* worker threads of a pool (BJXA_THREADS = total threads incl. the caller) */
inline unsigned
pool_threads(void)
{
	const char *e = getenv("BJXA_THREADS");
	if (e != NULL && *e != '\0') {
		const long v = strtol(e, NULL, 10);
		return v <= 1 ? 0u : (unsigned)std::min(v - 1, 63L);
	}
	/* the callers of a GPU box get a share of its cores: stay small */
	const unsigned hw = std::thread::hardware_concurrency();
	return std::min(hw > 1 ? hw - 1 : 0u, 15u);
}

}	/* namespace xa_pool */

#endif
