"""Writes tests/golden/ssz_vectors.json: the reference's own vectors for the
signing-root step in front of the hot path (include/tbls_ssz.h).

Sources (values transcribed from the reference test files, the deposit
vectors parsed from the reference's golden file when /root/reference is
present; the committed JSON is what the tests read):
  eth2util/hash_test.go:27-34                 SlotHashRoot(2)
  eth2util/types_test.go:27-36                SignedEpoch{Epoch: 2}.HashTreeRoot()
  core/validatorapi/validatorapi_test.go:230-289  TestSignAndVerify: domain,
      AttestationData root, SigningData root and the signature (sk = 1)
  eth2util/deposit/testdata/TestMarshalDepositData.golden  deposit message /
      data roots and signatures (fork 00001020, zero genesis validators root)
  eth2util/signing/signing_test.go:34-80      Teku ValidatorRegistration (root
      as recomputed in SURVEY.md §4, pinned by the signature)

Run from the repo root:  python tests/golden/make_ssz_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ssz_vectors.json")
REF_DEPOSIT = "/root/reference/eth2util/deposit/testdata/TestMarshalDepositData.golden"


def pad_to(b: bytes, n: int) -> bytes:  # validatorapi_test.go:326-332
    return b + bytes(n - len(b)) if len(b) <= n else b


def main():
    old = json.load(open(OUT)) if os.path.exists(OUT) else {}
    vec = {
        "slot_hash_root": [{"slot": 2, "root": "02" + "00" * 31}],
        "epoch_root": [{"epoch": 2, "root": "02" + "00" * 31}],
        "sign_and_verify_attestation": {
            "domain_type": "01000000", "fork_version": "64656666",
            "genesis_validators_root": (bytes([1, 2]) + bytes(30)).hex(),
            "domain": "0100000011b4296f38fa573d05f00854d452e120725b4d24b5587a472c6c4258",
            "slot": 999, "index": 0, "beacon_block_root": pad_to(b"blockRoot", 32).hex(),
            "source": {"epoch": 100, "root": "00" * 32}, "target": {"epoch": 200, "root": "00" * 32},
            "attestation_data_root": "eee68bd8e94662122695d04afa5fd5c30ae385c9f39d98aa840062f43221d0d0",
            "signing_root": "02bbdb88056d6cbafd6e94575540e74b8cf2c0f2c1b79b8e17e7b21ed1694305",
            # SecretFromBytes(padTo([]byte{1}, 32)): big-endian bytes 01 00 .. 00, i.e. 2^248
            "secret_key": (bytes([1]) + bytes(31)).hex(),
            "signature": "b6a60f8497bd328908be83634d045dd7a32f5e246b2c4031fc2f316983f362e36fc27fd3d6d5a2b15b4dbff"
                         "38804ffb10b1719b7ebc54e9cbf3293fd37082bc0fc91f79d70ce5b04ff13de3c8e10bb41305bfdbe921a43"
                         "792c12624f225ee865",
        },
        "validator_registration": {
            "fee_recipient": "000000000000000000000000000000000000dead", "gas_limit": 30000000,
            "timestamp": 1646092800,
            "pubkey": "86966350b672bd502bfbdb37a6ea8a7392e8fb7f5ebb5c5e2055f4ee168ebfab0fef63084f28c9f62c3ba71f825e527e",
            "root": "2c231b16a80337212ab1decde301bdb4383e74c0bf2f3439cc82542bf0f90fdd",
            "domain_type": "00000001", "fork_version": "00001020",
            # the signer is the secret share of signing_test.go:40 (its public
            # share), not the DV key inside the message
            "signer_secret": "345768c0245f1dc702df9e50e811002f61ebb2680b3d5931527ef59f96cbaf9b",
            "signer_pubkey": "9305c3b8cf2f4ee9c636b2e5bd60b730e4816840f01683bdcb75352451e553839c9173cd4212c08947443692dc48eaf7",
            "signature": "b101da0fc08addcc5d010ee569f6bbbdca049a5cb27efad231565bff2e3af504ec2bb87b11ed22843e9c1094f"
                         "1dfe51a0b2a5ad1808df18530a2f59f004032dbf6281ecf0fc3df86d032da5b9d32a3d282c05923de491381f"
                         "8f28c2863a00180",
        },
    }
    if os.path.exists(REF_DEPOSIT):
        deps = json.load(open(REF_DEPOSIT))
        vec["deposits"] = [{k: d[k] for k in ("pubkey", "withdrawal_credentials", "amount", "signature",
                                               "deposit_message_root", "deposit_data_root", "fork_version")}
                           for d in deps]
    else:
        vec["deposits"] = old["deposits"]
    json.dump(vec, open(OUT, "w"), indent=1)
    print("wrote", OUT, len(vec["deposits"]), "deposits")


if __name__ == "__main__":
    main()
