// dsp::Sink<T> lives in processor.h in this mirror (core/src/dsp/sink.h in the reference).
#pragma once
#include "processor.h"
