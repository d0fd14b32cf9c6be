# frozen_string_literal: true

# Batched delegators for Redis::Bloomfilter (lib/redis/bloomfilter.rb:61-73
# gains two siblings).  Drivers with a batch path (hip) get one call per batch;
# the ruby and lua drivers keep working through the per-key loop.
class Redis
  class Bloomfilter
    def insert_many(keys, expire = nil)
      expire ||= @options[:default_expire]
      return @driver.insert_many(keys, expire) if @driver.respond_to?(:insert_many)

      keys.each { |k| @driver.insert(k, expire) }
      nil
    end

    def include_many?(keys)
      return @driver.include_many?(keys) if @driver.respond_to?(:include_many?)

      keys.map { |k| @driver.include?(k) }
    end
  end
end
