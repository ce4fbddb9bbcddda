#!/bin/sh
# Regenerates the private-key fixtures of tests/test_sshkeys_native.py with
# this container's OpenSSH 8.9 / OpenSSL 3.0 (run once; the outputs are
# checked in so the tests need neither tool).  For every RSA/ECDSA key,
# <name>.expected.pem is what `ssh-keygen -p -m PEM -N ''` writes for it: the
# PKCS#1 / SEC1 PEM the in-process converter must reproduce byte for byte.
set -e
cd "$(dirname "$0")"
rm -f *.key *.pem *.pass
P=m2k-pass
kg() { ssh-keygen -q "$@" -C "m2k fixture"; }
kg -t rsa -b 2048 -N '' -f rsa_openssh.key
kg -t rsa -b 2048 -N "$P" -a 4 -f rsa_openssh_ctr.key
kg -t rsa -b 2048 -N "$P" -a 4 -Z aes256-cbc -f rsa_openssh_cbc.key
kg -t ecdsa -b 256 -N '' -f ec256_openssh.key
kg -t ecdsa -b 384 -N '' -f ec384_openssh.key
kg -t ecdsa -b 521 -N "$P" -a 4 -f ec521_openssh_ctr.key
kg -t ed25519 -N '' -f ed25519_openssh.key
kg -t dsa -N '' -f dsa_openssh.key
kg -t rsa -b 2048 -N '' -m PEM -f rsa_pkcs1.key
kg -t rsa -b 2048 -N "$P" -m PEM -f rsa_pkcs1_aes128.key
kg -t ecdsa -b 256 -N '' -m PEM -f ec256_sec1.key
kg -t ecdsa -b 384 -N "$P" -m PEM -f ec384_sec1_aes128.key
kg -t rsa -b 2048 -N '' -m PKCS8 -f rsa_pkcs8.key
kg -t ecdsa -b 256 -N '' -m PKCS8 -f ec256_pkcs8.key
kg -t dsa -N '' -m PEM -f dsa_pem.key
openssl rsa -in rsa_pkcs1.key -traditional -des3 -passout pass:$P -out rsa_pkcs1_des3.key 2>/dev/null
openssl rsa -in rsa_pkcs1.key -traditional -aes256 -passout pass:$P -out rsa_pkcs1_aes256.key 2>/dev/null
openssl ec -in ec256_sec1.key -aes192 -passout pass:$P -out ec256_sec1_aes192.key 2>/dev/null
openssl genpkey -algorithm ed25519 -out ed25519_pkcs8.key 2>/dev/null
rm -f *.pub
for k in *.key; do
  case $k in *ed25519*|*dsa*) continue ;; esac
  cp "$k" tmp.key
  chmod 600 tmp.key
  if grep -q ENCRYPTED "$k" || ssh-keygen -y -P '' -f "$k" >/dev/null 2>&1; then :; fi
  if ssh-keygen -y -P '' -f "$k" >/dev/null 2>&1; then old=''; else old=$P; fi
  ssh-keygen -q -p -m PEM -P "$old" -N '' -f tmp.key >/dev/null
  mv tmp.key "${k%.key}.expected.pem"
done
rm -f tmp.key*
