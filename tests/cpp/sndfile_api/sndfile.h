/* TEST INFRASTRUCTURE: the declarations of libsndfile's public API (sndfile.h, libsndfile
 * 1.x) that the .sdr dump uses -- libsndfile is not in this image.  Only for the compile
 * check that the drop-ins bind to libsndfile's own types when built with
 * -DDABGPU_HAVE_SNDFILE (tests/test_formats_cpu.py); nothing is linked against it. */
#ifndef SNDFILE_H
#define SNDFILE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
enum { SF_FORMAT_WAV = 0x010000, SF_FORMAT_PCM_16 = 0x0002 };
enum { SFM_READ = 0x10, SFM_WRITE = 0x20, SFM_RDWR = 0x30 };
typedef int64_t sf_count_t;
typedef struct SNDFILE_tag SNDFILE;
struct SF_INFO {
    sf_count_t frames;
    int samplerate, channels, format, sections, seekable;
};
typedef struct SF_INFO SF_INFO;
SNDFILE *sf_open(const char *path, int mode, SF_INFO *sfinfo);
sf_count_t sf_writef_short(SNDFILE *sndfile, const short *ptr, sf_count_t frames);
int sf_close(SNDFILE *sndfile);
#ifdef __cplusplus
}
#endif
#endif
