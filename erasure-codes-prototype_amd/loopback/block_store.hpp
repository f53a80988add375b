// Datanode block store adapters: the source and sink of the reference's data path.
//
// Datanode::store_data / access_data (project/src/datanode/datanode.cpp:64-169) keep a block either in
// an in-memory kv-map (IN_MEMORY build) or in a file ./storage/<port>/<block_id>.  Both backends are
// reproduced here, keyed by (datanode port, block id string), plus batched reads/writes that move many
// blocks between the store and one contiguous (ideally pinned) staging buffer, so a stripe batch can be
// handed to ecg_encode_batch_host / ecg_decode_batch_host without per-block copies.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace ecg_loopback {

class BlockStore {
public:
    virtual ~BlockStore() = default;
    // datanode.cpp:64-115 (insert / trunc-write).  Overwrites an existing key: the disk backend always
    // did (ios::trunc); the kv-map backend's std::unordered_map::insert would keep the OLD value, which
    // the reference never relies on (block ids are fresh, repairs go to other datanodes).
    virtual bool store_data(int port, const std::string& key, const char* value, size_t size) = 0;
    // datanode.cpp:117-169: reads exactly `size` bytes; false if the key does not exist.
    virtual bool access_data(int port, const std::string& key, char* out, size_t size) = 0;
    virtual bool remove_data(int port, const std::string& key) = 0;  // Datanode::delete (datanode.cpp:171+)
    virtual size_t count() = 0;

    // Batched adapters: block i of `keys` <-> staging + i * size.
    bool store_batch(const std::vector<int>& ports, const std::vector<std::string>& keys, const char* staging,
                     size_t size);
    bool access_batch(const std::vector<int>& ports, const std::vector<std::string>& keys, char* staging,
                      size_t size);
};

class KvBlockStore : public BlockStore {  // IN_MEMORY, no memcached/redis (datanode.cpp:89-97, 141-150)
public:
    bool store_data(int port, const std::string& key, const char* value, size_t size) override;
    bool access_data(int port, const std::string& key, char* out, size_t size) override;
    bool remove_data(int port, const std::string& key) override;
    size_t count() override;

private:
    std::mutex mu_;
    std::unordered_map<int, std::unordered_map<std::string, std::vector<char>>> nodes_;
};

class DiskBlockStore : public BlockStore {  // <root>/<port>/<block_id> (datanode.cpp:99-113, 151-165)
public:
    explicit DiskBlockStore(std::string root) : root_(std::move(root)) {}
    bool store_data(int port, const std::string& key, const char* value, size_t size) override;
    bool access_data(int port, const std::string& key, char* out, size_t size) override;
    bool remove_data(int port, const std::string& key) override;
    size_t count() override;
    std::string path(int port, const std::string& key) const;

private:
    std::string root_;
    std::mutex mu_;  // directory creation only
};

std::unique_ptr<BlockStore> make_block_store(const std::string& kind, const std::string& root);

}  // namespace ecg_loopback
