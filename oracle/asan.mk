# Sanitizer build of the CPU oracle (verdict round 5, item 7): the checker
# every parity claim rests on, with AddressSanitizer + UBSan, every finding fatal.  Host
# code only (tests/test_oracle_asan.py loads it into a child process with libasan
# preloaded); never built or run on the GPU box.
ASAN_FLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all
asan: _asan/liboracle_asan.so
_asan/liboracle_asan.so: anyseq_oracle.c
	mkdir -p _asan
	$(CC) $(ASAN_FLAGS) -fPIC -Wall -pthread -shared -o $@ $< -lpthread
.PHONY: asan
