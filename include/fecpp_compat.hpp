/*
 * fecpp_compat.hpp -- header-only drop-in for kcptube's `fecpp::fec_code` on top of libkfec.so.
 *
 * Replaces /root/reference/src/3rd_party/fecpp.hpp:14-89 with identical names and signatures, so
 * src/networks/connections.hpp:614 (`fecpp::fec_code fecc;`) and every caller (client.cpp:821/925,
 * server.cpp:956/1007, relay.cpp:1415/1454/1499, reset sites listed in SURVEY.md 3.3) compile unchanged.
 * Error behaviour is the reference's: the constructor and reset_martix throw std::invalid_argument on
 * a K/N violation (fecpp.cpp:431-432, 439-440); encode/decode return empty containers where the
 * reference returns {} (fecpp.cpp:497-498, 520-521, 550-551); decode throws std::invalid_argument where
 * invert_matrix would (fecpp.cpp:261, 303).  A missing GPU throws std::runtime_error: there is no CPU
 * path to fall back to.
 *
 * Link: -lkfec (kcptube_amd/libkfec.so).  See INTEGRATION.md.
 */
#ifndef FECPP_COMPAT_HPP_
#define FECPP_COMPAT_HPP_

#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "kfec.h"

namespace fecpp
{
	using std::uint8_t;
	using std::size_t;
	using byte = std::uint8_t;

#if defined(__i386__)|| defined(__amd64__) || defined(__x86_64__) || defined(_M_IX86) || defined(_M_X64) || defined(_M_AMD64)
#define FECPP_IS_X86
#endif

	class fec_code
	{
	public:
		fec_code() : K(0), N(0) {}

		fec_code(size_t K_arg, size_t N_arg) : K(0), N(0) { reset_martix(K_arg, N_arg); }

		fec_code(const fec_code &other) : K(0), N(0)
		{
			if (other.ctx) reset_martix(other.K, other.N);
		}

		fec_code &operator=(const fec_code &other)
		{
			if (this != &other)
			{
				if (other.ctx) reset_martix(other.K, other.N);
				else { ctx.reset(); K = N = 0; }
			}
			return *this;
		}

		fec_code(fec_code &&) noexcept = default;
		fec_code &operator=(fec_code &&) noexcept = default;

		void reset_martix(size_t K_arg, size_t N_arg)
		{
			if (K_arg == 0 || N_arg == 0 || K_arg > 256 || N_arg > 256 || K_arg > N_arg)
				throw std::invalid_argument("fec_code: violated 1 <= K <= N <= 256");
			int rc;
			if (ctx)
				rc = kfec_reset(ctx.get(), K_arg, N_arg);
			else
			{
				kfec_ctx *raw = nullptr;
				rc = kfec_create(K_arg, N_arg, &raw);
				if (rc == KFEC_OK) ctx.reset(raw);
			}
			raise(rc, "kfec_create");
			K = K_arg;
			N = N_arg;
		}

		size_t get_K() const { return K; }
		size_t get_N() const { return N; }

		std::vector<std::unique_ptr<uint8_t[]>> encode(const uint8_t input[], size_t data_length, size_t block_size) const
		{
			std::vector<std::unique_ptr<uint8_t[]>> redundant;
			if (!ctx || input == nullptr || block_size == 0) return redundant;
			const size_t R = N - K;
			std::unique_ptr<uint8_t[]> flat = std::make_unique<uint8_t[]>(R * block_size + 1);
			const int rc = kfec_encode(ctx.get(), input, data_length, block_size, flat.get());
			raise(rc, "kfec_encode");
			if (rc == KFEC_EMPTY) return redundant;
			for (size_t r = 0; r < R; ++r)
			{
				redundant.emplace_back(std::make_unique<uint8_t[]>(block_size));
				std::memcpy(redundant.back().get(), flat.get() + r * block_size, block_size);
			}
			return redundant;
		}

		std::map<size_t, std::vector<uint8_t>> decode(const std::map<size_t, const uint8_t *> &shares, size_t share_size) const
		{
			std::map<size_t, std::vector<uint8_t>> missing;
			if (!ctx || shares.size() < K) return missing;
			std::vector<size_t> ids;
			std::vector<const uint8_t *> ptrs;
			ids.reserve(shares.size());
			ptrs.reserve(shares.size());
			for (const auto &[id, p] : shares)
			{
				ids.push_back(id);
				ptrs.push_back(p);
			}
			std::vector<size_t> out_ids(K);
			std::vector<uint8_t> out(K * share_size + 1);
			size_t n_out = 0;
			const int rc = kfec_decode(ctx.get(), ids.data(), ptrs.data(), ids.size(), share_size, out_ids.data(), out.data(), &n_out);
			if (rc == KFEC_ESINGULAR) throw std::invalid_argument("singlar matrix");
			raise(rc, "kfec_decode");
			for (size_t t = 0; t < n_out; ++t)
				missing[out_ids[t]] = std::vector<uint8_t>(out.begin() + t * share_size, out.begin() + (t + 1) * share_size);
			return missing;
		}

		/* Beyond the reference interface: the device-resident batched path (include/kfec.h). */
		kfec_ctx *native_handle() const { return ctx.get(); }

	private:
		struct ctx_deleter { void operator()(kfec_ctx *c) const { kfec_destroy(c); } };
		size_t K, N;
		std::unique_ptr<kfec_ctx, ctx_deleter> ctx;

		static void raise(int rc, const char *what)
		{
			if (rc == KFEC_EINVAL) throw std::invalid_argument(std::string(what) + ": invalid argument");
			if (rc == KFEC_ENODEV) throw std::runtime_error(std::string(what) + ": no gfx950 device (no CPU fallback)");
			if (rc < 0) throw std::runtime_error(std::string(what) + ": HIP failure " + std::to_string(rc));
		}
	};

#if defined(FECPP_IS_X86)
	/* fecpp.hpp:83-85.  Declared so that code naming it still compiles; deliberately NOT defined: it is the
	 * reference's SSSE3 inner loop, nothing outside fecpp calls it, and this drop-in has no
	 * CPU compute path -- a use fails at link time instead of silently running on the host. */
	size_t addmul_ssse3(uint8_t z[], const uint8_t x[], uint8_t y, size_t size);
#endif
}

#endif
