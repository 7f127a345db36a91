// enc_cabac.h -- CABAC binary arithmetic encoder (host), the exact inverse of the
// decoder in ccmi_cabac.h.  Used by the .cool writer (enc_host.cpp).
//
// Behaviour follows the reference's TEncBinCABAC (coolchic/cpp/TEncBinCoderCABAC.cpp
// :58-340: start / finish / encodeBin / encodeBinEP / encodeBinsEP / encodeAlignedBinsEP /
// encodeBinTrm / writeOut) and the MSB-first OutputBitstream (BitStream.cpp:99-160), so
// that the bytes it emits are the reference encoder's bytes.  Errors (Exp-Golomb codes
// longer than 32 bins, which the reference exit()s on) are reported through `ok`.
#pragma once

#include <stdint.h>

#include <vector>

#include "ccmi_cabac.h"

namespace ccmi {

// MSB-first bit sink (OutputBitstream::write / writeAlignZero semantics).
struct BitSink {
    std::vector<uint8_t> bytes;
    uint64_t acc = 0; // pending bits, right-aligned
    int nacc = 0;     // < 8 between calls

    void put(uint32_t bits, int n)
    {
        if (n <= 0) return;
        const uint64_t m = n >= 32 ? 0xFFFFFFFFull : ((1ull << n) - 1);
        acc = (acc << n) | (bits & m);
        nacc += n;
        while (nacc >= 8) {
            nacc -= 8;
            bytes.push_back((uint8_t)(acc >> nacc));
        }
        acc &= (1ull << nacc) - 1;
    }
    void align_zero()
    {
        if (nacc > 0) bytes.push_back((uint8_t)(acc << (8 - nacc)));
        acc = 0;
        nacc = 0;
    }
};

struct CabacEnc {
    BitSink out;
    uint32_t low = 0, range = 510, buffered = 0xFF;
    int32_t nbuffered = 0, bits_left = 23;
    bool ok = true;

    void start()
    {
        low = 0;
        range = 510;
        buffered = 0xFF;
        nbuffered = 0;
        bits_left = 23;
    }

    // Carry propagation: the lead byte leaves `low`; 0xFF bytes wait for a possible carry.
    void write_out()
    {
        const uint32_t lead = low >> (24 - bits_left);
        bits_left += 8;
        low &= 0xFFFFFFFFu >> bits_left;
        if (lead == 0xFF) {
            ++nbuffered;
        } else if (nbuffered > 0) {
            const uint32_t carry = lead >> 8;
            out.put(buffered + carry, 8);
            buffered = lead & 0xFF;
            const uint32_t fill = (0xFF + carry) & 0xFF;
            for (; nbuffered > 1; --nbuffered) out.put(fill, 8);
        } else {
            nbuffered = 1;
            buffered = lead;
        }
    }

    // One bin against a model in state `st` (0..255; bit 7 = MPS).
    void bin_state(uint32_t st, uint32_t bin)
    {
        const uint32_t mps = st >> 7;
        const uint32_t q = mps ? st ^ 0xFFu : st;
        const uint32_t lps = (((q >> 2) * (range >> 5)) >> 1) + 4;
        range -= lps;
        if (bin != mps) {
            const uint32_t nb = lps_renorm(lps);
            bits_left -= (int32_t)nb;
            low += range;
            low <<= nb;
            range = lps << nb;
            if (bits_left < 12) write_out();
        } else if (range < 256) {
            bits_left -= 1;
            low <<= 1;
            range <<= 1;
            if (bits_left < 12) write_out();
        }
    }
    void bin_static(int idx, uint32_t bin)
    {
        Model m;
        m.init(idx);
        bin_state(m.state(), bin);
    }
    void bin_adaptive(Model &m, uint32_t bin)
    {
        bin_state(m.state(), bin);
        m.update(bin);
    }

    void ep(uint32_t bin)
    {
        low <<= 1;
        if (bin) low += range;
        if (--bits_left < 12) write_out();
    }

    void eps(uint32_t bins, int n)
    {
        if (range == 256) { // encodeAlignedBinsEP
            int rem = n;
            while (rem > 0) {
                const int take = rem < 8 ? rem : 8;
                const uint32_t v = (bins >> (rem - take)) & ((1u << take) - 1);
                low = (low << take) + (v << 8);
                rem -= take;
                bits_left -= take;
                if (bits_left < 12) write_out();
            }
            return;
        }
        while (n > 8) {
            n -= 8;
            const uint32_t pattern = bins >> n;
            low <<= 8;
            low += range * pattern;
            bins -= pattern << n;
            bits_left -= 8;
            if (bits_left < 12) write_out();
        }
        low <<= n;
        low += range * bins;
        bits_left -= n;
        if (bits_left < 12) write_out();
    }

    void expgolomb(uint32_t sym, uint32_t k)
    {
        uint32_t bins = 0;
        int n = 0;
        while (sym >= (1u << k)) {
            bins = 2 * bins + 1;
            ++n;
            sym -= 1u << k;
            ++k;
            if (k >= 31) {
                ok = false;
                return;
            }
        }
        bins = 2 * bins;
        ++n;
        bins = (bins << k) | sym;
        n += (int)k;
        if (n > 32) {
            ok = false;
            return;
        }
        eps(bins, n);
    }

    void trm(uint32_t bin)
    {
        range -= 2;
        if (bin) {
            low += range;
            low <<= 7;
            range = 2 << 7;
            bits_left -= 7;
        } else if (range >= 256) {
            return;
        } else {
            low <<= 1;
            range <<= 1;
            bits_left--;
        }
        if (bits_left < 12) write_out();
    }

    void finish()
    {
        if (low >> (32 - bits_left)) {
            out.put(buffered + 1, 8);
            for (; nbuffered > 1; --nbuffered) out.put(0x00, 8);
            low -= 1u << (32 - bits_left);
        } else {
            if (nbuffered > 0) out.put(buffered, 8);
            for (; nbuffered > 1; --nbuffered) out.put(0xFF, 8);
        }
        out.put(low >> 8, 24 - bits_left);
    }

    // Stream terminator used by every .cool sub-stream (ccencapi.cpp:148-151, :361-364):
    // terminating bin 1, flush, a stop bit, zero alignment.
    std::vector<uint8_t> &close()
    {
        trm(1);
        finish();
        out.put(1, 1);
        out.align_zero();
        return out.bytes;
    }
};

} // namespace ccmi
