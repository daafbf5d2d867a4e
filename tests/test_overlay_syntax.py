"""The drop-in overlay binds the reference's OWN block API.

INTEGRATION.md's recipe is literal here: the reference tree (core/src and the radio decoder module,
symlinked from /root/reference into a scratch directory) gets the overlay copied over it --
sdrpp_amd/dsp/gpu/dsp/** onto core/src/dsp/ and the IQFrontEnd drop-in onto
core/src/signal_path/iq_frontend.h (its iq_frontend.cpp is then dropped: the drop-in is header-only)
-- and the reference's own translation units that use the overlaid classes are compiled with
`g++ -fsyntax-only`:
  * a TU with every overlay header and explicit instantiations of the templates (FIR, DecimatingFIR,
    PowerDecimator, PolyphaseResampler, RationalResampler, FM, AM, SSB, AGC, DCBlocker, Deemphasis,
    FrequencyXlator): the overlay against the reference's Processor<I,O> (processor.h:42-73),
    stream<T> (stream.h:25-141) and block (block.h);
  * decoder_modules/radio/src/main.cpp: the radio module (demodulators/{wfm,nfm,am,usb,lsb,dsb,cw,
    raw}.h -> BroadcastFM, FM, AM, SSB, AGC, RationalResampler, Deemphasis) as SDR++ builds it;
  * core/src/signal_path/{signal_path,vfo_manager}.cpp: the callers of IQFrontEnd and RxVFO.
VOLK, FFTW and {fmt} are absent from this image, so tests/stubs/ holds declaration-only headers with
their published signatures: this proves that the overlay and its callers type-check against the
reference's interfaces -- signatures, never arithmetic. Nothing is linked or run, and nothing from
/root/reference is copied into the repository. Skipped where the reference tree is absent (GPU box).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
STUBS = os.path.join(ROOT, "tests", "stubs")
OVERLAY = os.path.join(ROOT, "sdrpp_amd", "dsp", "gpu")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "core", "src", "dsp")),
                                reason="reference tree not mounted (dev container only)")


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    t = tmp_path_factory.mktemp("ovl")
    core = t / "core_src"
    radio = t / "radio_src"
    subprocess.check_call(["cp", "-rs", os.path.join(REF, "core", "src"), str(core)])
    subprocess.check_call(["cp", "-rs", os.path.join(REF, "decoder_modules", "radio", "src"), str(radio)])
    placed = []
    for dp, _, fn in os.walk(os.path.join(OVERLAY, "dsp")):
        for f in fn:
            rel = os.path.relpath(os.path.join(dp, f), os.path.join(OVERLAY, "dsp"))
            dst = core / "dsp" / rel
            dst.parent.mkdir(parents=True, exist_ok=True)
            if dst.is_symlink() or dst.exists():
                dst.unlink()
            shutil.copyfile(os.path.join(dp, f), dst)
            placed.append(rel)
    dst = core / "signal_path" / "iq_frontend.h"
    dst.unlink()
    shutil.copyfile(os.path.join(OVERLAY, "signal_path", "iq_frontend.h"), dst)
    (core / "signal_path" / "iq_frontend.cpp").unlink()   # replaced by the header-only drop-in
    return t, sorted(placed)


def _syntax(t, src, extra=()):
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-w",
           "-I", str(t / "core_src"), "-I", str(t / "core_src" / "imgui"), "-I", str(t / "radio_src"),
           "-I", STUBS, "-I", os.path.join(ROOT, "include"), *extra, str(src)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    errs = [ln for ln in r.stderr.splitlines() if "error" in ln]
    assert r.returncode == 0, f"{src}: {len(errs)} errors\n" + "\n".join(errs[:40])


def test_overlay_placed_over_reference_counterparts(tree):
    """Every overlay header that replaces a reference header keeps that header's path."""
    _, placed = tree
    replaced = [p for p in placed if os.path.exists(os.path.join(REF, "core", "src", "dsp", p))]
    for p in ("channel/rx_vfo.h", "channel/frequency_xlator.h", "filter/fir.h", "filter/decimating_fir.h",
              "multirate/power_decimator.h", "multirate/rational_resampler.h", "multirate/polyphase_resampler.h",
              "demod/quadrature.h", "demod/fm.h", "demod/broadcast_fm.h", "demod/am.h", "demod/ssb.h",
              "loop/agc.h", "correction/dc_blocker.h", "filter/deephasis.h"):
        assert p in replaced, p


def test_overlay_headers_and_templates(tree):
    t, _ = tree
    src = t / "overlay_all.cpp"
    src.write_text("""
#include <dsp/channel/rx_vfo.h>
#include <dsp/channel/frequency_xlator.h>
#include <dsp/filter/fir.h>
#include <dsp/filter/decimating_fir.h>
#include <dsp/filter/deephasis.h>
#include <dsp/multirate/power_decimator.h>
#include <dsp/multirate/polyphase_resampler.h>
#include <dsp/multirate/rational_resampler.h>
#include <dsp/demod/quadrature.h>
#include <dsp/demod/fm.h>
#include <dsp/demod/broadcast_fm.h>
#include <dsp/demod/am.h>
#include <dsp/demod/ssb.h>
#include <dsp/loop/agc.h>
#include <dsp/correction/dc_blocker.h>
#include <dsp/signal_path/gpu_spectrum.h>
#include <signal_path/iq_frontend.h>
template class dsp::filter::FIR<dsp::complex_t, float>;
template class dsp::filter::FIR<float, float>;
template class dsp::filter::FIR<dsp::complex_t, dsp::complex_t>;
template class dsp::filter::DecimatingFIR<dsp::complex_t, float>;
template class dsp::filter::DecimatingFIR<float, float>;
template class dsp::multirate::PowerDecimator<dsp::complex_t>;
template class dsp::multirate::PolyphaseResampler<dsp::complex_t>;
template class dsp::multirate::RationalResampler<dsp::complex_t>;
template class dsp::multirate::RationalResampler<dsp::stereo_t>;
template class dsp::demod::FM<float>;
template class dsp::demod::FM<dsp::stereo_t>;
template class dsp::demod::AM<float>;
template class dsp::demod::AM<dsp::stereo_t>;
template class dsp::demod::SSB<float>;
template class dsp::demod::SSB<dsp::stereo_t>;
template class dsp::loop::AGC<float>;
template class dsp::loop::AGC<dsp::complex_t>;
template class dsp::correction::DCBlocker<dsp::complex_t>;
template class dsp::filter::Deemphasis<dsp::stereo_t>;
// the reference's base classes, exactly: Processor<I,O> with `out`, Processor's _in, block's run()
static_assert(std::is_base_of_v<dsp::Processor<dsp::complex_t, dsp::complex_t>, dsp::channel::RxVFO>);
static_assert(std::is_base_of_v<dsp::Processor<dsp::complex_t, float>, dsp::demod::Quadrature>);
static_assert(std::is_base_of_v<dsp::Processor<dsp::complex_t, dsp::stereo_t>, dsp::demod::BroadcastFM>);
static_assert(std::is_base_of_v<dsp::block, dsp::filter::FIR<dsp::complex_t, float>>);
int main() {
    dsp::stream<dsp::complex_t> in;
    dsp::channel::RxVFO vfo(&in, 61.44e6, 240000, 200000, 2.5e6);
    dsp::demod::BroadcastFM wfm(&vfo.out, 100000, 240000, true, false);
    vfo.setOffset(1e6);
    vfo.setBandwidth(150000);
    return vfo.out.read() + wfm.out.read();
}
""")
    _syntax(t, src)


def test_radio_module_compiles_against_overlay(tree):
    """decoder_modules/radio/src/main.cpp -- the radio module's own TU, every demodulator included."""
    t, _ = tree
    _syntax(t, t / "radio_src" / "main.cpp")


@pytest.mark.parametrize("tu", ["signal_path.cpp", "vfo_manager.cpp"])
def test_signal_path_compiles_against_overlay(tree, tu):
    """core/src/signal_path: the IQFrontEnd drop-in (header-only) and RxVFO under their callers."""
    t, _ = tree
    _syntax(t, t / "core_src" / "signal_path" / tu)
