// TEST INFRASTRUCTURE: gui.cpp:861-893 (set_dumping) as the reference writes it, against
// libsndfile's global names, compiled (not linked) with the drop-ins built -DDABGPU_HAVE_SNDFILE
#include "dabgpu_dropin.h"
// gui.cpp:861-893 as written, against libsndfile's global names
void set_dumping(dabgpu::ofdmProcessor *the_ofdmProcessor, const char *file) {
    SF_INFO sf_info;
    sf_info.samplerate = 2048000;
    sf_info.channels = 2;
    sf_info.format = SF_FORMAT_WAV | SF_FORMAT_PCM_16;
    SNDFILE *dumpfilePointer = sf_open(file, SFM_WRITE, &sf_info);
    the_ofdmProcessor->startDumping(dumpfilePointer);
    the_ofdmProcessor->stopDumping();
    sf_close(dumpfilePointer);
}
