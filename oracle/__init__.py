"""TEST INFRASTRUCTURE ONLY: CPU oracle for the checksum path (see tasx_oracle.h)."""
