// Mirror of dsp::sink::Handler<T> (core/src/dsp/sink/handler_sink.h:6-33): calls
// handler(data, count, ctx) for every batch; IQFrontEnd's FFT sink.
#pragma once
#include "../sink.h"

namespace dsp::sink {
template <class T>
class Handler : public Sink<T> {
    using base_type = Sink<T>;
public:
    Handler() {}
    Handler(stream<T>* in, void (*handler)(T* data, int count, void* ctx), void* ctx) { init(in, handler, ctx); }
    void init(stream<T>* in, void (*handler)(T* data, int count, void* ctx), void* ctx) {
        _handler = handler;
        _ctx = ctx;
        base_type::init(in);
    }
    void setHandler(void (*handler)(T* data, int count, void* ctx), void* ctx) {
        std::lock_guard<std::recursive_mutex> lk(base_type::ctrlMtx);
        base_type::tempStop();
        _handler = handler;
        _ctx = ctx;
        base_type::tempStart();
    }
    int run() override {
        int count = base_type::_in->read();
        if (count < 0) return -1;
        _handler(base_type::_in->readBuf, count, _ctx);
        base_type::_in->flush();
        return count;
    }

private:
    void (*_handler)(T* data, int count, void* ctx) = nullptr;
    void* _ctx = nullptr;
};
}  // namespace dsp::sink
