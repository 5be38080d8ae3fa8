/*
 * bpe_main.c -- command-line front end with the reference CLI's behaviour
 * (neofytr/LLMTokenizer main.c:3-25): train on <file_path> until the stop
 * rule, print the encoded text with print_text, free everything.
 * Built against the drop-in headers and linked with libbpe_amd.so.
 */
#include "../include/bpe.h"

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "Usage: %s <file_path>\n", argv[0]);
        return EXIT_FAILURE;
    }
    uint32_t *ids = NULL;
    size_t n = 0;
    dyn_arr_t *merges = compress(argv[1], &ids, &n);
    if (!merges) return EXIT_FAILURE;
    print_text(ids, (int)n);
    free(ids);
    dyn_arr_free(merges);
    return EXIT_SUCCESS;
}
