// Mirror of dsp::Processor<I,O> (core/src/dsp/processor.h:42-73): block with one input
// stream pointer and an owned output stream.
#pragma once
#include "block.h"

namespace dsp {
template <class I, class O>
class Processor : public block {
public:
    Processor() {}
    Processor(stream<I>* in) { init(in); }
    virtual ~Processor() {}
    virtual void init(stream<I>* in) {
        _in = in;
        registerInput(_in);
        registerOutput(&out);
        _block_init = true;
    }
    virtual void setInput(stream<I>* in) {
        assert(_block_init);
        std::lock_guard<std::recursive_mutex> lk(ctrlMtx);
        tempStop();
        unregisterInput(_in);
        _in = in;
        registerInput(_in);
        tempStart();
    }
    virtual int run() override = 0;
    stream<O> out;

protected:
    stream<I>* _in = nullptr;
};

// Mirror of dsp::Sink<T> (core/src/dsp/sink.h:6-36)
template <class T>
class Sink : public block {
public:
    Sink() {}
    Sink(stream<T>* in) { init(in); }
    virtual ~Sink() {}
    virtual void init(stream<T>* in) {
        _in = in;
        registerInput(_in);
        _block_init = true;
    }
    virtual void setInput(stream<T>* in) {
        assert(_block_init);
        std::lock_guard<std::recursive_mutex> lk(ctrlMtx);
        tempStop();
        unregisterInput(_in);
        _in = in;
        registerInput(_in);
        tempStart();
    }
    virtual int run() override = 0;

protected:
    stream<T>* _in = nullptr;
};
}  // namespace dsp
