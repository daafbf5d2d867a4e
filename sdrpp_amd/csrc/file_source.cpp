// file_source ingest on the host side of the boundary: the WAV container reader
// (source_modules/file_source/src/wavreader.h:34-226) and the worker's block framing
// (main.cpp:294-560: blocks of min(fs / 200, STREAM_BUFFER_SIZE) sample frames). The raw
// block bytes go to the device as they are; the sample conversion is the device converter
// (sdrgpu_convert_dev for two channels, sdrgpu_convert_mono_dev for one: I = Q = x).
//
// Reference behaviour kept on purpose:
//  * RIFF and RF64 ("ds64" chunk skipped, :119-133); fmt sizes < 16 or 17 rejected (:136);
//    WAVE_FORMAT_EXTENSIBLE mapped to PCM / IEEE_FLOAT by SubFormat.Data1 (:148-173), any other
//    SubFormat rejected; unknown chunks skipped (:183-187); the scan stops at "data" (:180-182).
//  * The sample region is [data offset, end of file): the data chunk's size field is not used,
//    so bytes of a chunk that follows "data" are read as samples too (getSampleCount :85-88,
//    readSamples :207-221). A partial frame at the end of the file is dropped.
//  * readSamples' bytesAvailable is computed as (fileSize - dataOffset) - tellg (:209), which
//    makes some reads near the end shorter than a block. It changes only where blocks split,
//    not the sample stream, and the spectrum / VFO path is block-split invariant, so blocks here
//    are always full except the last.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <algorithm>
#include "sdrgpu_internal.h"

using namespace sdrgpu;

struct sdrgpu_wav {
    FILE* f = nullptr;
    long long fileSize = 0, dataOffset = 0, pos = 0;   // pos: byte offset inside the sample region
    int format = 0, channels = 0, bits = 0, blockAlign = 0;
    unsigned sampleRate = 0;
};

namespace {
template <typename T> bool rd(FILE* f, T* v) { return std::fread(v, sizeof(T), 1, f) == 1; }

int wav_parse(sdrgpu_wav* w) {
    FILE* f = w->f;
    std::fseek(f, 0, SEEK_END);
    w->fileSize = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    char riff[4], type[4];
    uint32_t riffSize = 0;
    if (std::fread(riff, 1, 4, f) != 4 || !rd(f, &riffSize) || std::fread(type, 1, 4, f) != 4 ||
        !(std::memcmp(riff, "RIFF", 4) == 0 || std::memcmp(riff, "RF64", 4) == 0) || std::memcmp(type, "WAVE", 4) != 0) {
        set_error("wav: invalid WAV file");
        return SDRGPU_EARG;
    }
    bool fmt = false, data = false;
    while (std::ftell(f) < w->fileSize) {
        char id[4];
        uint32_t size = 0;
        if (std::fread(id, 1, 4, f) != 4 || !rd(f, &size)) break;
        if (std::memcmp(id, "ds64", 4) == 0) {
            uint64_t riff64, data64, count64;
            uint32_t table = 0;
            if (!rd(f, &riff64) || !rd(f, &data64) || !rd(f, &count64) || !rd(f, &table)) break;
            if (table > 0) std::fseek(f, (long)table * 12, SEEK_CUR);
            continue;
        } else if (std::memcmp(id, "fmt ", 4) == 0) {
            if (size < 16 || (size > 16 && size < 18)) { set_error("wav: invalid fmt chunk size %u", size); return SDRGPU_EARG; }
            uint16_t tag = 0, ch = 0, align = 0, bps = 0;
            uint32_t sr = 0, abps = 0;
            if (!rd(f, &tag) || !rd(f, &ch) || !rd(f, &sr) || !rd(f, &abps) || !rd(f, &align) || !rd(f, &bps)) break;
            if (size > 16) {
                uint16_t extra = 0;
                if (!rd(f, &extra)) break;
                if (tag == 0xFFFE && extra >= 22) {   // WAVE_FORMAT_EXTENSIBLE
                    uint16_t valid = 0, d2 = 0, d3 = 0;
                    uint32_t mask = 0, d1 = 0;
                    uint64_t d4 = 0;
                    if (!rd(f, &valid) || !rd(f, &mask) || !rd(f, &d1) || !rd(f, &d2) || !rd(f, &d3) || !rd(f, &d4)) break;
                    if (d1 == 1) tag = 1;
                    else if (d1 == 2) tag = 3;
                    else { set_error("wav: unknown format type for WAVE_FORMAT_EXTENSIBLE (%u)", d1); return SDRGPU_EARG; }
                } else {
                    std::fseek(f, extra, SEEK_CUR);
                }
            }
            w->format = tag; w->channels = ch; w->sampleRate = sr; w->blockAlign = align; w->bits = bps;
            fmt = true;
        } else if (std::memcmp(id, "data", 4) == 0) {
            data = true;
            break;
        } else {
            std::fseek(f, (long)size, SEEK_CUR);   // unknown chunk
        }
    }
    w->dataOffset = data ? std::ftell(f) : w->fileSize;
    if (!fmt || !data || w->blockAlign <= 0) { set_error("wav: no fmt or data chunk"); return SDRGPU_EARG; }
    // The reference's workers read the sample region as a packed stream of channels x bits/8-byte
    // frames (readSamples into inBuf, main.cpp:320-537) and use wBlockAlign only to count frames
    // (wavreader.h:85-88). A block align other than that frame size (padded or malformed) would
    // frame the samples differently from the converters, so such files are rejected; every read
    // below is sized by blockAlign == the packed frame size the callers allocate.
    if (w->bits <= 0 || (w->bits % 8) != 0 || w->channels <= 0 || w->blockAlign != w->channels * (w->bits / 8)) {
        set_error("wav: block align %d != channels (%d) x bytes per sample (%d bit)", w->blockAlign, w->channels, w->bits);
        return SDRGPU_EARG;
    }
    return SDRGPU_OK;
}
}  // namespace

extern "C" int sdrgpu_wav_open(sdrgpu_wav** out, const char* path) {
    if (!out || !path) { set_error("wav_open: null argument"); return SDRGPU_EARG; }
    *out = nullptr;
    auto* w = new sdrgpu_wav();
    w->f = std::fopen(path, "rb");
    if (!w->f) { set_error("wav_open: cannot open %s", path); delete w; return SDRGPU_EARG; }
    const int rc = wav_parse(w);
    if (rc < 0) { std::fclose(w->f); delete w; return rc; }
    *out = w;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_wav_info(sdrgpu_wav* w, int* format, int* channels, int* bits, double* sampleRate,
                               long long* sampleCount) {
    if (!w) { set_error("wav_info: null handle"); return SDRGPU_EARG; }
    if (format) *format = w->format;
    if (channels) *channels = w->channels;
    if (bits) *bits = w->bits;
    if (sampleRate) *sampleRate = w->sampleRate;
    if (sampleCount) *sampleCount = (w->fileSize - w->dataOffset) / w->blockAlign;
    return SDRGPU_OK;
}

// worker_1ch / worker_2ch: the converter for (format, bits), or an error for an unsupported one
extern "C" int sdrgpu_wav_kind(sdrgpu_wav* w) {
    if (!w) { set_error("wav_kind: null handle"); return SDRGPU_EARG; }
    if (w->channels != 1 && w->channels != 2) { set_error("wav: not supported channel count: %d", w->channels); return SDRGPU_EARG; }
    if (w->format == 3 && w->bits == 32) return SDRGPU_CONV_F32;   // IEEE float as it is
    if (w->format == 3 && w->bits == 64) return SDRGPU_CONV_F64;
    if (w->format == 1 && w->bits == 8) return SDRGPU_CONV_U8;
    if (w->format == 1 && w->bits == 16) return SDRGPU_CONV_I16;
    if (w->format == 1 && w->bits == 24) return SDRGPU_CONV_I24;
    if (w->format == 1 && w->bits == 32) return SDRGPU_CONV_I32;
    set_error("wav: not supported sample format: %d, %d bit", w->format, w->bits);
    return SDRGPU_EARG;
}

extern "C" int sdrgpu_wav_block_size(sdrgpu_wav* w) {
    if (!w) { set_error("wav_block_size: null handle"); return SDRGPU_EARG; }
    return std::max(1, (int)std::min<long long>(w->sampleRate / 200, 1000000));   // STREAM_BUFFER_SIZE
}

// next block of at most maxFrames sample frames, raw bytes into out (maxFrames * blockAlign bytes, where
// blockAlign = channels * bits / 8 is checked at open);
// returns the frames read, 0 at the end of the file
extern "C" int sdrgpu_wav_read(sdrgpu_wav* w, void* out, int maxFrames) {
    if (!w || (!out && maxFrames > 0) || maxFrames < 0) { set_error("wav_read: bad argument"); return SDRGPU_EARG; }
    const long long avail = (w->fileSize - w->dataOffset - w->pos) / w->blockAlign;
    const int n = (int)std::min<long long>(maxFrames, std::max(0LL, avail));
    if (n == 0) return 0;
    std::fseek(w->f, (long)(w->dataOffset + w->pos), SEEK_SET);
    const size_t got = std::fread(out, (size_t)w->blockAlign, (size_t)n, w->f);
    w->pos += (long long)got * w->blockAlign;
    return (int)got;
}

extern "C" int sdrgpu_wav_seek(sdrgpu_wav* w, long long frame) {   // WavReader::seek (:199-205)
    if (!w) { set_error("wav_seek: null handle"); return SDRGPU_EARG; }
    const long long count = (w->fileSize - w->dataOffset) / w->blockAlign;
    w->pos = std::max(0LL, std::min(frame, count)) * w->blockAlign;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_wav_close(sdrgpu_wav* w) {
    if (!w) return SDRGPU_OK;
    if (w->f) std::fclose(w->f);
    delete w;
    return SDRGPU_OK;
}
