// ccmi_cabac.h -- CABAC binary arithmetic decoder (HEVC/VVC style, as used by .cool
// bitstreams), usable from host code and from HIP device code.
//
// Behaviour follows the reference decoder's TDecBinCABAC (coolchic/cpp/
// TDecBinCoderCABAC.h:58-121, TDecBinCoderCABAC.cpp:64-178) and the VVC dual-rate
// probability model BinProbModel_Std (Contexts.h:84-176).  The byte source is a
// template parameter: a plain pointer on the host, a dword-window reader on the
// device.  Reads past the end of a stream return 0.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CCMI_HD __host__ __device__ __forceinline__
#else
#define CCMI_HD inline
#endif

namespace ccmi {

// Renormalisation shift after an LPS, indexed by lps_range >> 3 (Contexts.cpp:45-55).
CCMI_HD uint32_t lps_renorm(uint32_t lps)
{
    // 6,5,4,4,3,3,3,3,2 x8,1 x16 for lps>>3 in [0,32)
    const uint32_t i = lps >> 3;
    return i == 0 ? 6u : i == 1 ? 5u : i < 4 ? 4u : i < 8 ? 3u : i < 16 ? 2u : 1u;
}

// Adaptive binary model (two estimates at 10 and 14 bits; window DWS = 8).
struct Model {
    uint16_t s0, s1;
    CCMI_HD void init(int idx)
    {
        s0 = (uint16_t)((idx << 8) & 0x7FE0);
        s1 = (uint16_t)((idx << 8) & 0x7FFE);
    }
    CCMI_HD uint32_t state() const { return ((uint32_t)(s0 + s1) >> 8) & 0xFFu; }
    CCMI_HD void update(uint32_t bin)
    {
        // rate = DWS = 8 -> shifts 0 (first estimate) and 8 (second)
        s0 = (uint16_t)(s0 - (s0 & 0x7FE0));
        s1 = (uint16_t)(s1 - ((s1 >> 8) & 0x7FFE));
        if (bin) {
            s0 = (uint16_t)(s0 + (0x7FFFu & 0x7FE0));
            s1 = (uint16_t)(s1 + ((0x7FFFu >> 8) & 0x7FFE));
        }
    }
};

template <class Src>
struct Cabac {
    Src src;
    uint32_t range, value;
    int32_t bits_needed;

    CCMI_HD void start()
    {
        range = 510;
        value = src.next() << 8;
        value |= src.next();
        bits_needed = -8;
    }

    // Decode one bin for a model in state `st` (0..255).  Returns the bin.
    CCMI_HD uint32_t bin_state(uint32_t st)
    {
        uint32_t bin = st >> 7;
        const uint32_t q = bin ? st ^ 0xFFu : st;
        const uint32_t lps = (((q >> 2) * (range >> 5)) >> 1) + 4;
        range -= lps;
        const uint32_t scaled = range << 7;
        if (value < scaled) {
            if (range < 256) {
                range <<= 1;
                value <<= 1;
                if (++bits_needed >= 0) {
                    value += src.next() << bits_needed;
                    bits_needed -= 8;
                }
            }
        } else {
            const uint32_t nb = lps_renorm(lps);
            bin ^= 1u;
            value = (value - scaled) << nb;
            range = lps << nb;
            bits_needed += (int32_t)nb;
            if (bits_needed >= 0) {
                value += src.next() << bits_needed;
                bits_needed -= 8;
            }
        }
        return bin;
    }

    // Static (never updated) context initialised from state index idx (odd, 1..127).
    CCMI_HD uint32_t bin_static(int idx)
    {
        Model m;
        m.init(idx);
        return bin_state(m.state());
    }

    CCMI_HD uint32_t bin_adaptive(Model &m)
    {
        const uint32_t b = bin_state(m.state());
        m.update(b);
        return b;
    }

    CCMI_HD uint32_t ep()
    {
        value += value;
        if (++bits_needed >= 0) {
            value += src.next();
            bits_needed = -8;
        }
        const uint32_t scaled = range << 7;
        if (value >= scaled) {
            value -= scaled;
            return 1;
        }
        return 0;
    }

    CCMI_HD uint32_t eps(int n)
    {
        uint32_t bins = 0;
        if (range == 256) { // aligned fast path of the reference (decodeAlignedBinsEP)
            uint32_t rem = (uint32_t)n;
            while (rem > 0) {
                const uint32_t take = rem < 8 ? rem : 8;
                bins = (bins << take) | ((value >> (15 - take)) & ((1u << take) - 1));
                value = (value << take) & 0x7FFF;
                rem -= take;
                bits_needed += (int32_t)take;
                if (bits_needed >= 0) {
                    value |= src.next() << bits_needed;
                    bits_needed -= 8;
                }
            }
            return bins;
        }
        uint32_t rem = (uint32_t)n;
        while (rem > 8) {
            value = (value << 8) + (src.next() << (8 + bits_needed));
            uint32_t scaled = range << 15;
            for (int i = 0; i < 8; ++i) {
                bins += bins;
                scaled >>= 1;
                if (value >= scaled) {
                    bins++;
                    value -= scaled;
                }
            }
            rem -= 8;
        }
        bits_needed += (int32_t)rem;
        value <<= rem;
        if (bits_needed >= 0) {
            value += src.next() << bits_needed;
            bits_needed -= 8;
        }
        uint32_t scaled = range << (rem + 7);
        for (uint32_t i = 0; i < rem; ++i) {
            bins += bins;
            scaled >>= 1;
            if (value >= scaled) {
                bins++;
                value -= scaled;
            }
        }
        return bins;
    }

    CCMI_HD int32_t expgolomb(int k)
    {
        int32_t sym = 0;
        uint32_t bit = 1;
        while (bit) {
            bit = ep();
            sym += (int32_t)(bit << k);
            k++;
        }
        k--;
        if (k > 0) sym += (int32_t)eps(k);
        return sym;
    }
};

// Host byte source.
struct HostBytes {
    const uint8_t *p;
    uint32_t n, pos;
    CCMI_HD uint32_t next()
    {
        const uint32_t v = pos < n ? p[pos] : 0u;
        ++pos;
        return v;
    }
};

} // namespace ccmi
