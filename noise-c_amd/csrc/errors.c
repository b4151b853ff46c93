/*
 * errors.c — noise_strerror / noise_perror for the standalone library.
 *
 * The reference declares them in include/noise/protocol/errors.h and defines
 * them in src/protocol/errors.c:92-127; a program linked against this library
 * alone (no libnoiseprotocol) still gets them.  The message of each code is
 * part of that contract (errors.c:45-63) and is reproduced; codes without one
 * read "Unknown error 0x<code>".  When the reference's errors.c is linked
 * beside this library, its definitions take precedence.
 */
#include "noise_aead_hip.h"

#include <stdio.h>
#include <string.h>

static const char *err_text(int err)
{
    if (err == NOISE_ERROR_NONE) return "No error";
    if ((err >> 8) != 'E') return NULL;
    switch (err & 0xFF) {
    case 1: return "Out of memory";
    case 2: return "Unknown identifier";
    case 3: return "Unknown name";
    case 4: return "MAC failure";
    case 5: return "Not applicable";
    case 6: return "System error";
    case 7: return "Remote public key required";
    case 8: return "Local keypair required";
    case 9: return "Pre shared key required";
    case 10: return "Invalid length";
    case 11: return "Invalid parameter";
    case 12: return "Invalid state";
    case 13: return "Invalid nonce";
    case 14: return "Invalid private key";
    case 15: return "Invalid public key";
    case 16: return "Invalid format";
    case 17: return "Invalid signature";
    default: return NULL;
    }
}

void noise_perror(const char *s, int err)
{
    const char *t = err_text(err);
    if (!s) s = "(null)";
    if (t) fprintf(stderr, "%s: %s\n", s, t);
    else fprintf(stderr, "%s: Unknown error 0x%x\n", s, err);
}

int noise_strerror(int err, char *buf, size_t size)
{
    if (!buf || !size) return -1;
    const char *t = err_text(err);
    if (t) {
        const size_t n = strlen(t);
        const size_t k = n < size - 1 ? n : size - 1;
        memcpy(buf, t, k);
        buf[k] = '\0';
    } else {
        snprintf(buf, size, "Unknown error 0x%x", err);
    }
    return 0;
}
