// Mirror of dsp::stream<T> (core/src/dsp/stream.h:11-141): a writer/reader pair of
// STREAM_BUFFER_SIZE buffers handed over by swap(count) / read() / flush(), with
// stop flags that unblock either side. Same public interface; independent implementation.
#pragma once
#include <condition_variable>
#include <mutex>
#include "buffer/buffer.h"

#define STREAM_BUFFER_SIZE 1000000

namespace dsp {
class untyped_stream {
public:
    virtual ~untyped_stream() {}
    virtual bool swap(int size) { return false; }
    virtual int read() { return -1; }
    virtual void flush() {}
    virtual void stopWriter() {}
    virtual void clearWriteStop() {}
    virtual void stopReader() {}
    virtual void clearReadStop() {}
};

template <class T>
class stream : public untyped_stream {
public:
    stream() { setBufferSize(STREAM_BUFFER_SIZE); }
    virtual ~stream() { free(); }

    virtual void setBufferSize(int samples) {
        free();
        writeBuf = buffer::alloc<T>(samples);
        readBuf = buffer::alloc<T>(samples);
    }

    // writer: publish `size` samples of writeBuf; waits until the reader flushed the last batch
    bool swap(int size) override {
        std::unique_lock<std::mutex> lk(mtx);
        cv.wait(lk, [this] { return empty || wstop; });
        if (wstop) return false;
        std::swap(writeBuf, readBuf);
        count = size;
        empty = false;
        ready = true;
        cv.notify_all();
        return true;
    }
    // reader: wait for a batch (or stop); returns its size or -1
    int read() override {
        std::unique_lock<std::mutex> lk(mtx);
        cv.wait(lk, [this] { return ready || rstop; });
        return rstop ? -1 : count;
    }
    // reader: done with readBuf
    void flush() override {
        std::lock_guard<std::mutex> lk(mtx);
        ready = false;
        empty = true;
        cv.notify_all();
    }
    void stopWriter() override { std::lock_guard<std::mutex> lk(mtx); wstop = true; cv.notify_all(); }
    void clearWriteStop() override { std::lock_guard<std::mutex> lk(mtx); wstop = false; }
    void stopReader() override { std::lock_guard<std::mutex> lk(mtx); rstop = true; cv.notify_all(); }
    void clearReadStop() override { std::lock_guard<std::mutex> lk(mtx); rstop = false; }

    void free() {
        if (writeBuf) buffer::free(writeBuf);
        if (readBuf) buffer::free(readBuf);
        writeBuf = readBuf = nullptr;
    }

    T* writeBuf = nullptr;
    T* readBuf = nullptr;

private:
    std::mutex mtx;
    std::condition_variable cv;
    bool empty = true, ready = false, rstop = false, wstop = false;
    int count = 0;
};
}  // namespace dsp
