"""TEST INFRASTRUCTURE ONLY: CPU restatement of KungFu's host reduce and its
all-reduce schedule. Never imported by kungfu_amd/ (the product)."""
