// Datanode block store adapters: see block_store.hpp.
#include "block_store.hpp"

#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

namespace ecg_loopback {

bool BlockStore::store_batch(const std::vector<int>& ports, const std::vector<std::string>& keys,
                             const char* staging, size_t size) {
    if (ports.size() != keys.size()) return false;
    for (size_t i = 0; i < keys.size(); i++)
        if (!store_data(ports[i], keys[i], staging + i * size, size)) return false;
    return true;
}

bool BlockStore::access_batch(const std::vector<int>& ports, const std::vector<std::string>& keys, char* staging,
                              size_t size) {
    if (ports.size() != keys.size()) return false;
    for (size_t i = 0; i < keys.size(); i++)
        if (!access_data(ports[i], keys[i], staging + i * size, size)) return false;
    return true;
}

// ---------------------------------------------------------------- kv-map

bool KvBlockStore::store_data(int port, const std::string& key, const char* value, size_t size) {
    std::lock_guard<std::mutex> g(mu_);
    nodes_[port][key].assign(value, value + size);
    return true;
}

bool KvBlockStore::access_data(int port, const std::string& key, char* out, size_t size) {
    std::lock_guard<std::mutex> g(mu_);
    auto n = nodes_.find(port);
    if (n == nodes_.end()) return false;
    auto it = n->second.find(key);
    if (it == n->second.end() || it->second.size() < size) return false;
    memcpy(out, it->second.data(), size);
    return true;
}

bool KvBlockStore::remove_data(int port, const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    auto n = nodes_.find(port);
    return n != nodes_.end() && n->second.erase(key) > 0;
}

size_t KvBlockStore::count() {
    std::lock_guard<std::mutex> g(mu_);
    size_t c = 0;
    for (auto& n : nodes_) c += n.second.size();
    return c;
}

// ---------------------------------------------------------------- disk

std::string DiskBlockStore::path(int port, const std::string& key) const {
    return root_ + "/" + std::to_string(port) + "/" + key;
}

bool DiskBlockStore::store_data(int port, const std::string& key, const char* value, size_t size) {
    const std::string dir = root_ + "/" + std::to_string(port);
    {
        std::lock_guard<std::mutex> g(mu_);
        mkdir(root_.c_str(), S_IRWXU);
        if (access(dir.c_str(), F_OK) == -1 && mkdir(dir.c_str(), S_IRWXU) != 0) return false;
    }
    FILE* f = fopen(path(port, key).c_str(), "wb");
    if (!f) return false;
    const bool ok = fwrite(value, 1, size, f) == size;
    return fclose(f) == 0 && ok;
}

bool DiskBlockStore::access_data(int port, const std::string& key, char* out, size_t size) {
    FILE* f = fopen(path(port, key).c_str(), "rb");
    if (!f) return false;
    const bool ok = fread(out, 1, size, f) == size;
    fclose(f);
    return ok;
}

bool DiskBlockStore::remove_data(int port, const std::string& key) { return unlink(path(port, key).c_str()) == 0; }

size_t DiskBlockStore::count() {
    size_t c = 0;
    DIR* d = opendir(root_.c_str());
    if (!d) return 0;
    while (dirent* e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        DIR* s = opendir((root_ + "/" + e->d_name).c_str());
        if (!s) continue;
        while (dirent* f = readdir(s))
            if (f->d_name[0] != '.') c++;
        closedir(s);
    }
    closedir(d);
    return c;
}

std::unique_ptr<BlockStore> make_block_store(const std::string& kind, const std::string& root) {
    if (kind == "kv") return std::make_unique<KvBlockStore>();
    if (kind == "disk") return std::make_unique<DiskBlockStore>(root);
    return nullptr;
}

}  // namespace ecg_loopback
