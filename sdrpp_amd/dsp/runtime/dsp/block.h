// Mirror of dsp::block (core/src/dsp/block.h:11-130): one worker thread per block that
// loops run() until it returns < 0; start/stop and the nesting tempStop/tempStart used to
// park the worker while parameters change.
#pragma once
#include <algorithm>
#include <cassert>
#include <mutex>
#include <thread>
#include <vector>
#include "stream.h"
#include "types.h"

namespace dsp {
class generic_block {
public:
    virtual ~generic_block() {}
    virtual void start() {}
    virtual void stop() {}
    virtual int run() { return -1; }
};

class block : public generic_block {
public:
    virtual ~block() {
        if (_block_init) stop();
        _block_init = false;
    }
    void start() override {
        assert(_block_init);
        std::lock_guard<std::recursive_mutex> lk(ctrlMtx);
        if (running) return;
        running = true;
        doStart();
    }
    void stop() override {
        assert(_block_init);
        std::lock_guard<std::recursive_mutex> lk(ctrlMtx);
        if (!running) return;
        doStop();
        running = false;
    }
    void tempStart() {
        std::lock_guard<std::recursive_mutex> lk(ctrlMtx);
        if (tempStopDepth == 0 || --tempStopDepth > 0) return;
        if (tempStopped) {
            doStart();
            tempStopped = false;
        }
    }
    void tempStop() {
        std::lock_guard<std::recursive_mutex> lk(ctrlMtx);
        if (tempStopDepth++ > 0) return;
        if (running && !tempStopped) {
            doStop();
            tempStopped = true;
        }
    }
    virtual int run() override = 0;

protected:
    void workerLoop() {
        while (run() >= 0) {}
    }
    virtual void doStart() { workerThread = std::thread(&block::workerLoop, this); }
    virtual void doStop() {
        for (auto* s : inputs) s->stopReader();
        for (auto* s : outputs) s->stopWriter();
        if (workerThread.joinable()) workerThread.join();
        for (auto* s : inputs) s->clearReadStop();
        for (auto* s : outputs) s->clearWriteStop();
    }
    void registerInput(untyped_stream* s) { inputs.push_back(s); }
    void unregisterInput(untyped_stream* s) { inputs.erase(std::remove(inputs.begin(), inputs.end(), s), inputs.end()); }
    void registerOutput(untyped_stream* s) { outputs.push_back(s); }
    void unregisterOutput(untyped_stream* s) { outputs.erase(std::remove(outputs.begin(), outputs.end(), s), outputs.end()); }

    bool _block_init = false;
    std::recursive_mutex ctrlMtx;
    std::vector<untyped_stream*> inputs, outputs;
    bool running = false, tempStopped = false;
    int tempStopDepth = 0;
    std::thread workerThread;
};
}  // namespace dsp
